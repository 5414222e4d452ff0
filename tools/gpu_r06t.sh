#!/bin/bash
# Round 6: the bs = 3 tile table (FEM_ASM_HASH3: the reference row's deltas hashed, matching rows look their
# positions up; build/var_h3): bit-identity tests, 10M elastic / Poisson kernel stats against the default build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VL=$PWD/cuda-powered-mesh-handling-and-iterative-solvers_amd/build
for v in h3 cur; do
  FEM355_LIB=$VL/var_$v/libfem355.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
      -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_matfree.py -m gpu \
      > gpurun_out/pytest_t_$v.log 2>&1; rc=$?; echo "== $v tests rc=$rc"; tail -1 gpurun_out/pytest_t_$v.log
  [ $rc -ne 0 ] && { tail -40 gpurun_out/pytest_t_$v.log; exit $rc; }
done
for K in elastic poisson; do
  KIND=$K bash tools/asm_ab.sh cur h3 > gpurun_out/asm_t_$K.log 2>&1 || exit $?
  rm -rf gpurun_out/asmv_t_$K; mv gpurun_out/asmv gpurun_out/asmv_t_$K
  for d in gpurun_out/asmv_t_$K/*/; do echo "== $K $d"; python3 tools/kstats.py $d/run_kernel_stats.csv 3 | grep asm_tet4; done
done
