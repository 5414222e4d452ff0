#!/bin/bash
# Round 6: ke_row1 software-pipelined over its passes (FEM_KE_PIPE1=1, build/var_pipe1) vs one pass at a time (default):
# the stored-matrix assembly parity tests, then tools/mass_tile_probe.py with each library, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B=$PWD/cuda-powered-mesh-handling-and-iterative-solvers_amd/build
FEM355_LIB=$B/var_pipe1/libfem355.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "fused_stiffness_mass or scalar_mass_and_bs1 or config4 or mass or tile_assembly_bit" \
  > gpurun_out/r06zj_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r06zj_tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/r06zj_tests.log | head -20; exit $rc; }
for rep in 1 2; do
  for v in def pipe1; do
    if [ $v = def ]; then unset FEM355_LIB; else export FEM355_LIB=$B/var_$v/libfem355.so; fi
    timeout -k 10 200 python tools/mass_tile_probe.py > gpurun_out/r06zj_${v}_$rep.json 2>gpurun_out/r06zj_${v}_$rep.err || exit $?
    python -c "
import json;d=json.load(open('gpurun_out/r06zj_${v}_$rep.json'))
print('$v', {k:(round(x['mass']['ms_median'],3), round(x['stiffness']['ms_median'],3), x['mass']['bits_sum']%100000) for k,x in d.items()})"
  done
done
echo zj-done
