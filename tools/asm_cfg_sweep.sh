#!/bin/bash
# assembly A/B on the 10M cube: default kernels, the wave-per-row value kernels (FEM355_ASM_ROWS) and the radix-sort
# incidence (FEM355_INC_RADIX); the value sums must be the same bits in every configuration
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for kind in poisson elastic; do
  for v in "FEM355_NONE=1" "FEM355_ASM_ROWS=1" "FEM355_INC_RADIX=1"; do
    echo "$kind $v $(env $v timeout -k 10 120 python3 tools/assemble_only.py --n 119 --kind $kind --reps 3 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print([round(x["graph_ms"],3) for x in d], [round(x["assemble_ms"],3) for x in d], len(set(x["vals_bits"] for x in d)), d[-1]["vals_bits"])')" || exit 1
  done
done
