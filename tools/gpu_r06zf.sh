#!/bin/bash
# Round 6: tile height of the bs = 1 stored-element-matrix assembly (k_assemble_ke_tile1, FEM_KE_R1 16 / 8 / 4):
# tools/mass_tile_probe.py with each library, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B=$PWD/cuda-powered-mesh-handling-and-iterative-solvers_amd/build
for rep in 1 2; do
  for v in def r1_8 r1_4; do
    if [ $v = def ]; then unset FEM355_LIB; else export FEM355_LIB=$B/var_$v/libfem355.so; fi
    timeout -k 10 200 python tools/mass_tile_probe.py > gpurun_out/r06zf_${v}_$rep.json 2>gpurun_out/r06zf_${v}_$rep.err || exit $?
    python -c "
import json;d=json.load(open('gpurun_out/r06zf_${v}_$rep.json'))
print('$v', {k:(round(x['mass']['ms_median'],3), round(x['stiffness']['ms_median'],3), x['mass']['bits_sum']%100000) for k,x in d.items()})"
  done
done
echo zf-done
