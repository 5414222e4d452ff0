#!/bin/bash
# Round 6: LDS-atomic sweep adds in the accumulator assembly (FEM_ACC_ATOM, build/var_atom): bit-identity tests on the
# variant, then 10M elastic and Poisson assembly kernel stats against the default build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VL=$PWD/cuda-powered-mesh-handling-and-iterative-solvers_amd/build
for v in atom acc3 pdpp; do
  FEM355_LIB=$VL/var_$v/libfem355.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
      -p no:cacheprovider tests/test_gpu_parity.py -m gpu -k "tile or solver_layout or elastic or poisson or assembl" \
      > gpurun_out/pytest_o_$v.log 2>&1; rc=$?; echo "== $v tests rc=$rc"; tail -1 gpurun_out/pytest_o_$v.log
  [ $rc -ne 0 ] && { tail -40 gpurun_out/pytest_o_$v.log; exit $rc; }
done
for K in elastic poisson; do
  KIND=$K bash tools/asm_ab.sh atom acc3 pdpp > gpurun_out/asm_o_$K.log 2>&1 || exit $?
  rm -rf gpurun_out/asmv_o_$K; mv gpurun_out/asmv gpurun_out/asmv_o_$K
  for d in gpurun_out/asmv_o_$K/*/; do echo "== $K $d"; python3 tools/kstats.py $d/run_kernel_stats.csv 3 | grep asm_tet4; done
done
