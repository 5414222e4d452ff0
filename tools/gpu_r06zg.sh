#!/bin/bash
# Round 6: the repeated-node check of the stored-K_e assemblies (ke_row1 / ke_row3) by cross-lane reads (default)
# vs the reload loop (FEM_KE_DUPLOAD=1, build/var_dupload): assembly parity tests, tools/mass_tile_probe.py with each
# library alternating (and ke_row1 adds as LDS atomics, build/var_atom1), then the configs[4] mixed companion.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B=$PWD/cuda-powered-mesh-handling-and-iterative-solvers_amd/build
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "fused_stiffness_mass or packed_symmetric or scalar_mass_and_bs1 or config4 or element_row_assembly or tile_assembly_bit or solver_layout_elastic or solid_ke or mass" \
  > gpurun_out/r06zg_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r06zg_tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/r06zg_tests.log | head -20; exit $rc; }
for rep in 1 2; do
  for v in def dupload atom1; do
    if [ $v = def ]; then unset FEM355_LIB; else export FEM355_LIB=$B/var_$v/libfem355.so; fi
    timeout -k 10 200 python tools/mass_tile_probe.py > gpurun_out/r06zg_${v}_$rep.json 2>gpurun_out/r06zg_${v}_$rep.err || exit $?
    python -c "
import json;d=json.load(open('gpurun_out/r06zg_${v}_$rep.json'))
print('$v', {k:(round(x['mass']['ms_median'],3), round(x['stiffness']['ms_median'],3), x['mass']['bits_sum']%100000) for k,x in d.items()})"
  done
done
unset FEM355_LIB
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --elastic 0 --config1 0 --dof-passes 3 \
    > gpurun_out/r06zg_mixed_$rep.json 2>gpurun_out/r06zg_mixed_$rep.err || exit $?
  python -c "
import json;d=json.loads(open('gpurun_out/r06zg_mixed_$rep.json').read().strip().splitlines()[-1])['mixed']
print('mixed', round(d['set_ms'],3), {k:(round(d[k]['job_ms'],3), {a:(round(b,3) if b else b) for a,b in d[k]['stage_ms'].items()}) for k in ('c3d8','c3d6','c3d10')})"
done
echo zg-done
