#!/bin/bash
# Counter passes for the element-chunk operator (run on the GPU box): tools/mf_probe.py under rocprofv3 -- kernel
# stats, SQ wait / VALU / LDS counters, FETCH_SIZE, WRITE_SIZE; each --pmc pass its own run (no trace domains).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/pmc_mf}
ARGS=${MF_ARGS:-"--n 119 --no-assembled --iters 10"}
mkdir -p $O
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES"
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- python3 tools/mf_probe.py $ARGS > $O/trace.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $SQ -f csv -d $O/sq -o run -- python3 tools/mf_probe.py $ARGS > $O/sq.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $O/fetch -o run -- python3 tools/mf_probe.py $ARGS > $O/fetch.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $O/write -o run -- python3 tools/mf_probe.py $ARGS > $O/write.log 2>&1 || exit $?
tail -1 $O/trace.log
