#!/bin/bash
# Round 6: the distributed persistent kernels on ranks emulated on one GPU (tools/dist_persist_check.py) at the
# N = 8 rank share of the 10M cube (n = 59): single-reduction vs pipelined DIST builds, 1 and 2 ranks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for gv in "" "--gv"; do
    timeout -k 10 300 python tools/dist_persist_check.py --n 59 --ranks 1 2 --iters 5 --time-iters 2000 $gv \
      > gpurun_out/r06z8_${rep}${gv}.json 2>&1 || exit $?
    python -c "
import json;d=json.loads(open('gpurun_out/r06z8_${rep}${gv}.json').read().strip().splitlines()[-1])
print('gv' if d['gv'] else 'sr', {P: (round(d[P]['us_per_it'],2), d[P]['solve']['iters'], d[P]['solve']['x_rel']) for P in ('P1','P2')}, d['single'])"
  done
done
