#!/bin/bash
# One GPU-box pass: GPU tests, smoke, bench. Each GPU step has its own time limit; a fault/abort/timeout stops
# the script (exit codes >= 124 or signals); ordinary test failures (exit 1) do not stop the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" >> gpurun_out/steps.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >> gpurun_out/steps.log
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ $rc -gt 128 ]; then
    echo "fatal rc=$rc in $name; stopping"; tail -20 "gpurun_out/$name.log"; exit $rc
  fi
  return $rc
}
rm -f gpurun_out/steps.log
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
  step pytest_gpu 1100 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider --durations=20
  step smoke 300 python __graft_entry__.py smoke
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 900 python bench.py ${BENCH_ARGS}
fi
tail -5 gpurun_out/pytest_gpu.log 2>/dev/null; tail -3 gpurun_out/smoke.log 2>/dev/null; tail -2 gpurun_out/bench.log 2>/dev/null
cat gpurun_out/steps.log
