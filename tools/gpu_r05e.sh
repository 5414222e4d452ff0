#!/bin/bash
# Round-5 GPU pass E: the element-chunk walk with rotated prefetch records -- parity tests, K1 timing, phase-skip build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_matfree.py tests/test_dist_gpu.py -m gpu -k "matfree or chunk or mf" \
    > gpurun_out/pytest_e.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_e.log; [ $rc -ne 0 ] && exit $rc
for v in def prof3; do
  L=""; [ $v != def ] && L=FEM355_LIB=$PWD/cuda-powered-mesh-handling-and-iterative-solvers_amd/build/var_$v/libfem355.so
  env $L timeout -k 10 200 python tools/mf_probe.py --n 119 --iters 50 > gpurun_out/mfprof_e_$v.log 2>&1
  rc=$?; echo "== $v rc=$rc"; grep '^{' gpurun_out/mfprof_e_$v.log | tail -1 | head -c 900; echo; [ $rc -ge 124 ] && exit $rc
done
exit 0
