#!/bin/bash
# Round 6: configs[4] stiffness + mass in one pass (fem_assemble_from_ke_mass_sl): parity tests, then the mixed
# companion with the fused and the split global assemblies, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "fused_stiffness_mass or packed_symmetric or scalar_mass_and_bs1 or config4 or isoparametric_mass" \
  > gpurun_out/r06zd_tests.log 2>&1; rc=$?; tail -4 gpurun_out/r06zd_tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/r06zd_tests.log | head -20; exit $rc; }
for rep in 1 2; do
  for m in fused split; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --elastic 0 --config1 0 \
      --dof-passes 3 --mixed-km $m > gpurun_out/r06zd_mixed_${m}_$rep.json 2>gpurun_out/r06zd_mixed_${m}_$rep.err || exit $?
    python -c "
import json;d=json.loads(open('gpurun_out/r06zd_mixed_${m}_$rep.json').read().strip().splitlines()[-1])['mixed']
print('$m', round(d['set_ms'],3), {k:(round(d[k]['job_ms'],3), {a:(round(b,3) if b else b) for a,b in d[k]['stage_ms'].items()}) for k in ('c3d8','c3d6','c3d10')})"
  done
done
echo zd-done
