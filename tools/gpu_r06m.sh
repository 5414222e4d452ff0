#!/bin/bash
# Round 6 probes: (1) the LDS-staged update slot sums (FEM_MF_QLDS) A/B and the K1 phase-skip timing builds
# (FEM_MF_PROF 1/2/3, wrong results) against the default on the 10M
# elastic cube; (2) the resident grid of the chunk kernels capped (FEM355_MF_GRID_CAP) at the N = 8 rank share, where
# 2,450 chunks leave ~2.4 per workgroup of the default grid (world-1 RCCL line, element-chunk operator).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_mf_ab.sh qlds0,prof1,prof2,prof3 r06l || exit $?
for cap in 0 512 256; do
  if [ $cap = 0 ]; then unset FEM355_MF_GRID_CAP; else export FEM355_MF_GRID_CAP=$cap; fi
  timeout -k 10 300 python bench.py --force-dist --n 59 --steps 200 --warmup 20 --no-cpu-baseline --mixed 0 \
    --reference-api 0 --matfree 1 > gpurun_out/r06m_n59_cap$cap.json 2>gpurun_out/r06m_n59_cap$cap.err || exit $?
  python -c "
import json;d=json.loads(open('gpurun_out/r06m_n59_cap$cap.json').read().strip().splitlines()[-1]);m=d['elasticity']['element_rccl']['matfree']
print('cap $cap', round(m['ms_per_step']*1e3,2), {a: round(b*1e3,2) for a,b in m['kernel_ms'].items()})"
done
