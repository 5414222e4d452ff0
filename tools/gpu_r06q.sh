#!/bin/bash
# Round 6: g_b shared over DPP in the elastic sweep (FEM_ACC_GDPP, build/var_gdpp): bit-identity tests, kernel stats
# against the default; SQ counters of the default build's elastic value kernel (two passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VL=$PWD/cuda-powered-mesh-handling-and-iterative-solvers_amd/build
for v in gdpp; do
  FEM355_LIB=$VL/var_$v/libfem355.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
      -p no:cacheprovider tests/test_gpu_parity.py -m gpu -k "tile or solver_layout or elastic or poisson or assembl" \
      > gpurun_out/pytest_q_$v.log 2>&1; rc=$?; echo "== $v tests rc=$rc"; tail -1 gpurun_out/pytest_q_$v.log
  [ $rc -ne 0 ] && { tail -40 gpurun_out/pytest_q_$v.log; exit $rc; }
done
KIND=elastic bash tools/asm_ab.sh gdpp > gpurun_out/asm_q.log 2>&1 || exit $?
rm -rf gpurun_out/asmv_q; mv gpurun_out/asmv gpurun_out/asmv_q
for d in gpurun_out/asmv_q/*/; do echo "== $d"; python3 tools/kstats.py $d/run_kernel_stats.csv 3 | grep asm_tet4; done
KIND=elastic bash tools/pmc_asm_kind.sh || exit $?
echo pmc-done
