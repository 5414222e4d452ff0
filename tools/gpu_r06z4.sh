#!/bin/bash
# Round 6: the pipelined kernel's one-slot build with 4 lane pairs in flight (FEM_GV_U1=4, no VGPR spills) against
# the default 8 (5 VGPRs spilled): tools/gv_probe.py at n = 55 and 59, alternating builds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/cuda-powered-mesh-handling-and-iterative-solvers_amd/build
for rep in 1 2; do
for n in 55 59; do
  for v in def gu4; do
    L=$PWD/cuda-powered-mesh-handling-and-iterative-solvers_amd/lib/libfem355.so; [ $v != def ] && L=$V/var_$v/libfem355.so
    echo "== $v"; FEM355_LIB=$L timeout -k 10 120 python tools/gv_probe.py --n $n --iters 500 2>&1 | grep pipelined= || exit $?
  done
done
done
