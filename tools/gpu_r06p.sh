#!/bin/bash
# Round 6: the default build after the accumulator sweep change and the per-partition distributed form: distributed,
# element-chunk and parity GPU tests, world-1 RCCL lines at the rank share (gather form) and at 10M (gather-free),
# and the 10M elastic / Poisson value kernels' stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py tests/test_gpu_matfree.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06p_tests.log 2>&1 || { tail -30 gpurun_out/r06p_tests.log; exit 1; }
tail -2 gpurun_out/r06p_tests.log
for n in 59 119; do
  timeout -k 10 400 python bench.py --force-dist --n $n --steps 200 --warmup 20 --no-cpu-baseline \
    --mixed 0 --reference-api 0 > gpurun_out/r06p_dist_n$n.json 2>gpurun_out/r06p_dist_n$n.err || exit $?
  python -c "
import json;d=json.loads(open('gpurun_out/r06p_dist_n$n.json').read().strip().splitlines()[-1]);m=d['elasticity']['element_rccl']['matfree']
print('n$n', round(m['ms_per_step']*1e3,2), {a: round(b*1e3,2) for a,b in m['kernel_ms'].items()}, m['solve_iters'])"
done
for K in elastic poisson; do
  KIND=$K bash tools/asm_ab.sh > gpurun_out/asm_p_$K.log 2>&1 || exit $?
  rm -rf gpurun_out/asmv_p_$K; mv gpurun_out/asmv gpurun_out/asmv_p_$K
  python3 tools/kstats.py gpurun_out/asmv_p_$K/def/run_kernel_stats.csv 3 | grep asm_tet4
done
