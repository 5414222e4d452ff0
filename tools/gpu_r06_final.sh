#!/bin/bash
# Round-6 end-of-round evidence on the final tree, in two calls (each under gpurun's 1200 s):
#   bash tools/gpu_r06_final.sh a : GPU tests + smoke + the default bench line (tools/gpu_round.sh)
#   bash tools/gpu_r06_final.sh b : the bench at the driver's settings (--steps 20 --warmup 5), rocprofv3 kernel
#                                   stats + FETCH_SIZE / WRITE_SIZE passes of the Poisson bench (separate runs), and
#                                   the element-chunk operator's kernel stats + SQ / FETCH / WRITE passes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
case ${1:-a} in
a)
  bash tools/gpu_round.sh all || exit $?
  ;;
b)
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r06z_bench_20steps.json 2>gpurun_out/r06z_bench_20steps.err || exit $?
  tail -c 300 gpurun_out/r06z_bench_20steps.json; echo
  OUT=gpurun_out/prof_z PROF_ARGS="--steps 100 --warmup 10 --no-cpu-baseline --elastic 0 --mixed 0 --reference-api 0" \
    bash tools/profile_round.sh > /dev/null || exit $?
  OUT=gpurun_out/pmc_mf_z bash tools/pmc_mf.sh || exit $?
  ;;
esac
echo final-$1-done
