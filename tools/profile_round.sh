#!/bin/bash
# rocprofv3 evidence for the bench workload (run on the GPU box):
#   pass 1: --kernel-trace --stats           -> per-kernel average durations (compare with bench.py's live events)
#   pass 2: --pmc FETCH_SIZE (+kernel-trace) -> HBM read bytes per dispatch  (gfx950: x2 for wide streams)
#   pass 3: --pmc WRITE_SIZE (+kernel-trace) -> HBM write bytes per dispatch
# No sys/runtime/hip/hsa/memory-copy traces are combined with --pmc.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof}
mkdir -p $OUT
export FEM355_PK_COOP=0   # rocprofv3 segfaults at exit after a cooperative launch (the timed launches are plain)
ARGS=${PROF_ARGS:-"--steps 100 --warmup 10 --no-cpu-baseline"}
set -o pipefail
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1 || exit $?
find $OUT -name "*.csv" | head -50
