#!/bin/bash
# Round 6: ke_row3's adds as LDS atomics (FEM_KE_ATOM=1, default) vs read-modify-write (build/var_keatom0): the
# stored-K_e assembly bit-identity tests, then the configs[4] mixed companion (fused and split global assemblies)
# with each library, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/cuda-powered-mesh-handling-and-iterative-solvers_amd/build/var_keatom0/libfem355.so
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "fused_stiffness_mass or packed_symmetric or scalar_mass_and_bs1 or config4 or element_row_assembly or tile_assembly_bit or solver_layout_elastic or solid_ke" \
  > gpurun_out/r06ze_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r06ze_tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/r06ze_tests.log | head -20; exit $rc; }
for rep in 1 2; do
  for lib in atom rmw; do
    if [ $lib = rmw ]; then export FEM355_LIB=$V; else unset FEM355_LIB; fi
    for m in fused split; do
      timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --elastic 0 --config1 0 \
        --dof-passes 3 --mixed-km $m > gpurun_out/r06ze_${lib}_${m}_$rep.json 2>gpurun_out/r06ze_${lib}_${m}_$rep.err || exit $?
      python -c "
import json;d=json.loads(open('gpurun_out/r06ze_${lib}_${m}_$rep.json').read().strip().splitlines()[-1])['mixed']
print('$lib $m', round(d['set_ms'],3), {k:(round(d[k]['job_ms'],3), {a:(round(b,3) if b else b) for a,b in d[k]['stage_ms'].items() if a.startswith('assemble')}) for k in ('c3d8','c3d6','c3d10')})"
    done
  done
done
echo ze-done
