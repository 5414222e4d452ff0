#!/bin/bash
# Round-5 GPU pass G: the 512-thread / two-lanes-per-node chunk walk (FEM_MF_W512 build) -- matrix-free parity under
# it, then K1 timing of the default walk, its phase-skip builds and the W512 build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VL=$PWD/cuda-powered-mesh-handling-and-iterative-solvers_amd/build
FEM355_LIB=$VL/var_w512/libfem355.so timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    -p no:cacheprovider tests/test_gpu_matfree.py -m gpu > gpurun_out/pytest_g_w512.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_g_w512.log; [ $rc -ge 124 ] && exit $rc
for v in def w512 prof1 prof2; do
  L=""; [ $v != def ] && L=FEM355_LIB=$VL/var_$v/libfem355.so
  env $L timeout -k 10 200 python tools/mf_probe.py --n 119 --no-assembled --iters 50 > gpurun_out/mfprof_g_$v.log 2>&1
  rc=$?; echo "== $v rc=$rc"; grep '^{' gpurun_out/mfprof_g_$v.log | tail -1 | head -c 700; echo; [ $rc -ge 124 ] && exit $rc
done
exit 0
