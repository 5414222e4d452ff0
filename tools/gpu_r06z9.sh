#!/bin/bash
# Round 6: the multi-process path of the pipelined DIST build (bench.py --gpus 2 --pipelined 1, both ranks on this
# GPU) and the single-reduction one, via tests/test_gpu_dist_persist.py's bench tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_persist.py -x -v --timeout 400 --timeout-method thread \
  -p no:cacheprovider -k "bench_two_ranks" > gpurun_out/r06z9_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed|Error|assert" gpurun_out/r06z9_tests.log | tail -20
exit $rc
