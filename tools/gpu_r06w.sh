#!/bin/bash
# Round 6: the pipelined persistent Jacobi-PCG (FEM_TUNE_PK_GV, csrc/pcg_persist_gv.hpp): its GPU tests, then the
# Poisson bench line at the 1M-tet configs[1] cube (n = 55) and at the N = 8 rank share of the 10M cube (n = 59),
# single-reduction and pipelined, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipelined.py -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r06w_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|assert" gpurun_out/r06w_tests.log | tail -25
[ $rc -ne 0 ] && exit $rc
A="--elastic 0 --mixed 0 --reference-api 0 --no-cpu-baseline --dof-passes 1"
for n in 55 59; do
  for pl in 0 1; do
    timeout -k 10 300 python bench.py --n $n --steps 500 --warmup 50 --pipelined $pl $A > gpurun_out/r06w_n${n}_p$pl.json 2>gpurun_out/r06w_n${n}_p$pl.err || exit $?
    python -c "
import json;d=json.loads(open('gpurun_out/r06w_n${n}_p$pl.json').read().strip().splitlines()[-1])
print('n$n pipelined=$pl', d.get('pipelined'), round(d['value']), 'it/s', round(d['ms_per_step']*1e3,2), 'us/step', round(d['kernel_ms']['persist_iteration']*1e3,2), 'us/it', 'dofs/s', round(d['dofs_per_s']/1e6,1), 'M', 'iters', d['solve_iters'])"
  done
done
