#!/bin/bash
# round-3 rocprofv3 evidence: the bench's Poisson line and the elasticity system at the driver's 20 / 5 steps,
# each as kernel-trace stats + separate FETCH_SIZE and WRITE_SIZE passes (tools/profile_round.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/prof_p PROF_ARGS="--steps 20 --warmup 5 --no-cpu-baseline --elastic 0" bash tools/profile_round.sh || exit $?
OUT=gpurun_out/prof_e PROF_ARGS="--kind elastic --steps 20 --warmup 5 --no-cpu-baseline" bash tools/profile_round.sh || exit $?
