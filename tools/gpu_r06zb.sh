#!/bin/bash
# Round 6: the pipelined kernel with GV launched with the single-reduction kernel LDS size (FEM_GV_BIGLDS=1,
# build/var_biglds) against the default: pipelined tests, then tools/gv_probe.py alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/cuda-powered-mesh-handling-and-iterative-solvers_amd/build
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipelined.py -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r06zb_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r06zb_tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/r06zb_tests.log | head; exit $rc; }
for rep in 1 2; do
  for v in def biglds; do
    L=$PWD/cuda-powered-mesh-handling-and-iterative-solvers_amd/lib/libfem355.so; [ $v != def ] && L=$V/var_$v/libfem355.so
    for n in 55 59; do
      echo "== $v"; FEM355_LIB=$L timeout -k 10 120 python tools/gv_probe.py --n $n --iters 1000 2>&1 | grep pipelined= || exit $?
    done
  done
done
