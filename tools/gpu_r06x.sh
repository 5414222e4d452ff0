#!/bin/bash
# Round 6: timing probes of the pipelined persistent kernel (tools/gv_probe.py): the default build, no barrier wait
# (FEM_GV_PROBE=1), neither the barrier nor the m-flag wait (=3); n = 55 (1M) and 59 (10M rank share).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/cuda-powered-mesh-handling-and-iterative-solvers_amd/build
timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -x -q -k "16bit_positions" --timeout 100 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r06x_tests.log 2>&1; echo "width test rc=$?"; tail -1 gpurun_out/r06x_tests.log
for n in 55 59; do
  for v in def gvp1 gvp3; do
    L=$PWD/cuda-powered-mesh-handling-and-iterative-solvers_amd/lib/libfem355.so; [ $v != def ] && L=$V/var_$v/libfem355.so
    echo "== $v"; FEM355_LIB=$L timeout -k 10 120 python tools/gv_probe.py --n $n --iters 500 2>&1 | grep -v amdgpu.ids || exit $?
  done
done
