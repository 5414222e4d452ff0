#!/bin/bash
# Round 6: the default bench line at the driver's settings with the configs[1] companion (single-reduction and
# pipelined persistent kernels at 1M tets).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r06z2_bench_20steps.json 2>gpurun_out/r06z2_bench_20steps.err || exit $?
python -c "
import json;d=json.loads(open('gpurun_out/r06z2_bench_20steps.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step']); print(json.dumps(d.get('config1'), indent=1))"
