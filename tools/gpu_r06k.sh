#!/bin/bash
# Round 6: distributed paths after the chunk-kernel LDS padding, the fixed-count slot loads and the 16-byte-lane update (k_cg1_update):
# distributed GPU tests, then world-1 RCCL lines at the N = 8 rank share and at 10M.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py tests/test_gpu_matfree.py -x -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r06k_tests.log 2>&1 || { tail -30 gpurun_out/r06k_tests.log; exit 1; }
tail -2 gpurun_out/r06k_tests.log
for n in 59 119; do
  timeout -k 10 400 python bench.py --force-dist --n $n --steps 200 --warmup 20 --no-cpu-baseline --mixed 0 \
    --reference-api 0 > gpurun_out/r06k_dist_world1_n$n.json 2>gpurun_out/r06k_dist_world1_n$n.err || exit $?
done
