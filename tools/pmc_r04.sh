#!/bin/bash
# Round-4 counter passes (run on the GPU box), each --pmc pass its own rocprofv3 run (no trace domains combined):
#   assembly value kernels (tools/assemble_only.py, 10M cube, poisson + elastic): SQ wait / VALU / LDS counters,
#   FETCH_SIZE, WRITE_SIZE;  BASELINE configs[4] mixed set (tools/bench_mixed.py): kernel stats, FETCH_SIZE,
#   WRITE_SIZE of k_iso_ke and the stored-K_e assembly kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/pmc_r04}
mkdir -p $O
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES"
PART=${1:-all}
if [ "$PART" = all ] || [ "$PART" = asm ]; then
  for kind in poisson elastic; do
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $SQ -f csv -d $O/asm_${kind}_sq -o run -- python3 tools/assemble_only.py --n 119 --kind $kind --reps 2 > $O/asm_${kind}_sq.log 2>&1 || exit $?
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $O/asm_${kind}_fetch -o run -- python3 tools/assemble_only.py --n 119 --kind $kind --reps 2 > $O/asm_${kind}_fetch.log 2>&1 || exit $?
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $O/asm_${kind}_write -o run -- python3 tools/assemble_only.py --n 119 --kind $kind --reps 2 > $O/asm_${kind}_write.log 2>&1 || exit $?
  done
fi
if [ "$PART" = all ] || [ "$PART" = mixed ]; then
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats -f csv -d $O/mixed_trace -o run -- python3 tools/bench_mixed.py --cpu-sample 0 > $O/mixed_trace.log 2>&1 || exit $?
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $O/mixed_fetch -o run -- python3 tools/bench_mixed.py --cpu-sample 0 > $O/mixed_fetch.log 2>&1 || exit $?
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $O/mixed_write -o run -- python3 tools/bench_mixed.py --cpu-sample 0 > $O/mixed_write.log 2>&1 || exit $?
fi
find $O -name "*.csv" | head -40
