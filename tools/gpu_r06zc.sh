#!/bin/bash
# Round 6: host wait of the timed persistent launch -- the end event polled (default) against hipEventSynchronize
# (FEM355_EVSYNC=block): tools/launch_overhead.py and the Poisson bench line at the driver's 20 / 5 steps, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for m in spin block; do
    E=""; [ $m = block ] && E=block
    echo "== launch_overhead $m"
    FEM355_EVSYNC=$E timeout -k 10 180 python tools/launch_overhead.py --ks 1 20 100 --reps 7 \
      > gpurun_out/r06zc_overhead_${m}_$rep.json || exit $?
    python -c "import json;d=json.load(open('gpurun_out/r06zc_overhead_${m}_$rep.json'));print({k:(round(v['wall_us'],1),round(v['event_us'],1),round(v['host_us'],1)) for k,v in d['rows_per_k'].items()}, d['fit'])"
  done
done
for rep in 1 2; do
  for m in spin block; do
    E=""; [ $m = block ] && E=block
    FEM355_EVSYNC=$E timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --elastic 0 --mixed 0 \
      --config1 0 --dof-passes 1 > gpurun_out/r06zc_bench20_${m}_$rep.json 2>gpurun_out/r06zc_bench20_${m}_$rep.err || exit $?
    python -c "import json;d=json.loads(open('gpurun_out/r06zc_bench20_${m}_$rep.json').read().strip().splitlines()[-1]);print('$m', round(d['value'],1), d['ms_per_step'], d['kernel_ms'])"
  done
done
echo zc-done
