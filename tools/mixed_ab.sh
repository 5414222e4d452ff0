#!/bin/bash
# BASELINE configs[4] mixed-family bench, A/B of environment knobs (run on the GPU box): each line is one
# tools/bench_mixed.py run (GPU work only) with the knob set, e.g.  bash tools/mixed_ab.sh "" "FEM355_KE_SELLW=1"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/mixed_ab}
mkdir -p $O
i=0
for cfg in "$@"; do
  i=$((i + 1))
  echo "== [$cfg]" >> $O/ab.log
  timeout -k 10 200 env $cfg python3 tools/bench_mixed.py --cpu-sample 0 > $O/run$i.log 2>&1 || exit $?
  tail -1 $O/run$i.log >> $O/ab.log
done
cat $O/ab.log
