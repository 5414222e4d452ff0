#!/bin/bash
# Round 6: the pipelined kernel, current library vs the one built from commit 557fab8 (same source of the kernel):
# box or build? tools/gv_probe.py, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/cuda-powered-mesh-handling-and-iterative-solvers_amd/build
for rep in 1 2; do
  for v in def old; do
    L=$PWD/cuda-powered-mesh-handling-and-iterative-solvers_amd/lib/libfem355.so; [ $v != def ] && L=$V/var_$v/libfem355.so
    echo "== $v"; FEM355_LIB=$L timeout -k 10 120 python tools/gv_probe.py --n 55 --iters 1000 2>&1 | grep pipelined= || exit $?
  done
done
