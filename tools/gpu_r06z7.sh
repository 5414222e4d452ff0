#!/bin/bash
# Round 6: the pipelined DIST build on emulated ranks (tests/test_gpu_pipelined.py), then the single-reduction DIST
# tests (tests/test_gpu_dist_persist.py) for regressions.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipelined.py -x -v -s --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r06z7_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed|iterations|Error|assert" gpurun_out/r06z7_tests.log | tail -30
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_persist.py -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r06z7_dist.log 2>&1; rc=$?
tail -2 gpurun_out/r06z7_dist.log
exit $rc
