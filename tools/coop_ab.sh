#!/bin/bash
# timed Poisson line at the driver's 20 / 5 steps: cooperative persistent launch (default) vs plain launch
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/coop
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --elastic 0 --no-cpu-baseline --dof-passes 1 > gpurun_out/coop/coop$i.json 2> gpurun_out/coop/coop$i.err || exit $?
  FEM355_PK_COOP=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --elastic 0 --no-cpu-baseline --dof-passes 1 > gpurun_out/coop/plain$i.json 2> gpurun_out/coop/plain$i.err || exit $?
done
for f in gpurun_out/coop/*.json; do echo "$f $(python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(round(d['value']), round(d['ms_per_step']*1e3,2), round(d['kernel_ms']['persist_iteration']*1e3,2))")"; done
