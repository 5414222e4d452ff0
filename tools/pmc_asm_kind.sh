#!/bin/bash
# SQ counters (two passes) of every assembly kernel of the 10M cube: KIND=poisson|elastic (default poisson)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
KIND=${KIND:-poisson}
O=gpurun_out/pmc_$KIND
mkdir -p $O
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES"
C2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C1 -f csv -d $O/c1 -o run -- python3 tools/assemble_only.py --n 119 --kind $KIND --reps 2 > $O/c1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C2 -f csv -d $O/c2 -o run -- python3 tools/assemble_only.py --n 119 --kind $KIND --reps 2 > $O/c2.log 2>&1 || exit $?
