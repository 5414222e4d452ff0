#!/bin/bash
# Round 6: the pipelined persistent kernel with the early arrival (default) -- its tests, then tools/gv_probe.py for
# the default build, the late-arrival build (FEM_GV_EARLY=0) and the no-barrier-wait timing build (FEM_GV_PROBE=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/cuda-powered-mesh-handling-and-iterative-solvers_amd/build
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipelined.py -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r06y_tests.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r06y_tests.log | tail -3
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/r06y_tests.log | head; exit $rc; }
for n in 55 59; do
  for v in def gvlate gvp1; do
    L=$PWD/cuda-powered-mesh-handling-and-iterative-solvers_amd/lib/libfem355.so; [ $v != def ] && L=$V/var_$v/libfem355.so
    echo "== $v"; FEM355_LIB=$L timeout -k 10 120 python tools/gv_probe.py --n $n --iters 500 2>&1 | grep -v amdgpu.ids || exit $?
  done
done
