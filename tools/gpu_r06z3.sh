#!/bin/bash
# Round 6: the pipelined kernel's GPU tests with their measured errors printed (incl. configs[1] vs the oracle).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipelined.py -x -v -s --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r06z3_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed|iterations|vs oracle|Error|assert" gpurun_out/r06z3_tests.log | tail -30
exit $rc
