#!/bin/bash
# Round 6: run-to-run spread of the pipelined vs single-reduction persistent kernels (tools/gv_probe.py), with the
# box's partition modes and clocks recorded.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rocm-smi --showcomputepartition --showmemorypartition 2>/dev/null | grep -iE "partition" | head -4
rocm-smi --showclocks 2>/dev/null | grep -E "fclk|mclk|socclk" | head -3
hostname
for rep in 1 2; do
  for n in 55 59; do
    timeout -k 10 120 python tools/gv_probe.py --n $n --iters 1000 2>&1 | grep pipelined= || exit $?
  done
done
