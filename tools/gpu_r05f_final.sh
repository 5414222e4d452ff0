#!/bin/bash
# Round-5 end-of-round rocprofv3 evidence (after the value-kernel search and stream-order changes): kernel stats + FETCH_SIZE / WRITE_SIZE passes of the
# Poisson bench run (separate runs), and the element-chunk operator's kernel stats + SQ counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
BASE="--no-cpu-baseline --elastic 0 --mixed 0 --reference-api 0"
OUT=gpurun_out/prof_f PROF_ARGS="--steps 100 --warmup 10 $BASE" bash tools/profile_round.sh > /dev/null || exit $?
grep '^{' gpurun_out/prof_f/trace.log | tail -1 | head -c 400; echo
OUT=gpurun_out/pmc_mf_f bash tools/pmc_mf.sh || exit $?
