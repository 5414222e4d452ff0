#!/bin/bash
# assembly value-kernel configurations (FEM355_ASM_CFG / FEM355_ASM_TILE / FEM355_ASM_ROWS) on the 10M cube
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for kind in poisson elastic; do
  for v in "FEM355_ASM_CFG=0" "FEM355_ASM_CFG=1" "FEM355_ASM_CFG=2" "FEM355_ASM_TILE=1" "FEM355_ASM_ROWS=1"; do
    echo "$kind $v $(env $v timeout -k 10 120 python3 tools/assemble_only.py --n 119 --kind $kind --reps 3 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print([round(x["assemble_ms"],3) for x in d], len(set(x["vals_bits"] for x in d)))')" || exit 1
  done
done
