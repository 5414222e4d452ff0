#!/bin/bash
# SQ / TA counters of the 10M elastic assembly kernel (k_asm_tet4_acc<3>), three passes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmc_el3
mkdir -p $O
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES"
C3="TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum"
C2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAIT_INST_LDS"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C1 -f csv -d $O/def1 -o run -- python3 tools/assemble_only.py --n 119 --kind elastic --reps 2 > $O/def1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C2 -f csv -d $O/def2 -o run -- python3 tools/assemble_only.py --n 119 --kind elastic --reps 2 > $O/def2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C3 -f csv -d $O/def3 -o run -- python3 tools/assemble_only.py --n 119 --kind elastic --reps 2 > $O/def3.log 2>&1 || exit $?

