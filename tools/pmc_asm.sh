#!/bin/bash
# SQ counters of the assembly kernels (tile vs row kernels), one --pmc pass per configuration
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmc_asm
mkdir -p $O
CTR="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES"
for kind in poisson elastic; do
  for rows in 0 1; do
    if [ $rows = 1 ]; then export FEM355_ASM_ROWS=1; else unset FEM355_ASM_ROWS; fi
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTR -f csv -d $O/${kind}_$rows -o run -- python3 tools/assemble_only.py --n 119 --kind $kind --reps 2 > $O/${kind}_$rows.log 2>&1 || exit $?
  done
done
