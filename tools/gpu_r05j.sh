#!/bin/bash
# Round-5 GPU pass J: the elastic tile kernel's accumulators transposed ([row][slot], FEM_ACC_T builds with row
# padding 1 / 4 / 8): bit-identity tests under each build, then the 10M elastic assembly kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VL=$PWD/cuda-powered-mesh-handling-and-iterative-solvers_amd/build
for v in acct1 acct4 acct8; do
  FEM355_LIB=$VL/var_$v/libfem355.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
      -p no:cacheprovider tests/test_gpu_parity.py -m gpu -k "tile or solver_layout_elastic or elastic" \
      > gpurun_out/pytest_j_$v.log 2>&1; rc=$?; echo "== $v tests rc=$rc"; tail -1 gpurun_out/pytest_j_$v.log
  [ $rc -ne 0 ] && exit $rc
done
KIND=elastic bash tools/asm_ab.sh acct1 acct4 acct8 > gpurun_out/asm_j.log 2>&1 || exit $?
rm -rf gpurun_out/asmv_j; mv gpurun_out/asmv gpurun_out/asmv_j
for d in gpurun_out/asmv_j/*/; do echo "== $d"; python3 tools/kstats.py $d/run_kernel_stats.csv 3 | grep asm_tet4; done
