#!/bin/bash
# Round 6: packed symmetric K_e (configs[4] internal path) parity tests + the mixed bench line; rocprofv3 kernel stats
# (csv) of the world-1 RCCL element-partition line at the N = 8 rank share (n = 59).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "packed or isoparametric or tile_assembly" -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06d_tests.log 2>&1 || { tail -30 gpurun_out/r06d_tests.log; exit 1; }
tail -2 gpurun_out/r06d_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_scale_parity.py -k "config4" -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06d_tests4.log 2>&1 || { tail -30 gpurun_out/r06d_tests4.log; exit 1; }
tail -2 gpurun_out/r06d_tests4.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --elastic 0 --reference-api 0 \
  > gpurun_out/r06d_bench_mixed.json 2>gpurun_out/r06d_bench_mixed.err || exit $?
FEM355_PK_COOP=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06d_prof_n59 -o run -- \
  python3 bench.py --force-dist --n 59 --steps 200 --warmup 20 --no-cpu-baseline --mixed 0 --reference-api 0 \
  > gpurun_out/r06d_dist_world1_n59.json 2>gpurun_out/r06d_dist_world1_n59.err || exit $?
find gpurun_out/r06d_prof_n59 -name "*stats.csv"
