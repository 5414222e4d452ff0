#!/bin/bash
# Quick GPU check: selected tests (-k expression in $1) then an optional command ($2); each step time-limited.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "$1" > gpurun_out/quick_tests.log 2>&1
rc=$?
tail -15 gpurun_out/quick_tests.log
[ $rc -ne 0 ] && exit $rc
if [ -n "$2" ]; then
  timeout -k 10 600 bash -c "$2" > gpurun_out/quick_cmd.log 2>&1
  rc=$?
  tail -30 gpurun_out/quick_cmd.log
  exit $rc
fi
