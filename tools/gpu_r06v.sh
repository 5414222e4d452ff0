#!/bin/bash
# Round 6: L2 prefetch of the next SpMV's first slice under the persistent kernel's grid barrier (FEM_PK_PF,
# build/var_pf): persistent-schedule GPU tests on the variant, then the Poisson bench line (200 and 20 steps) for
# the default build and the variant, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/cuda-powered-mesh-handling-and-iterative-solvers_amd/build/var_pf/libfem355.so
FEM355_LIB=$V timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_gpu_scale_parity.py tests/test_dist_gpu.py -m gpu -k "persist or metric or scale or dist" \
  > gpurun_out/pytest_v.log 2>&1 || { tail -30 gpurun_out/pytest_v.log; exit 1; }
tail -1 gpurun_out/pytest_v.log
A="--elastic 0 --mixed 0 --reference-api 0 --no-cpu-baseline"
for rep in 1 2; do
  for v in def pf; do
    L=$PWD/cuda-powered-mesh-handling-and-iterative-solvers_amd/lib/libfem355.so; [ $v = pf ] && L=$V
    for st in 200 20; do
      W=20; [ $st = 20 ] && W=5
      FEM355_LIB=$L timeout -k 10 300 python bench.py --steps $st --warmup $W $A > gpurun_out/r06v_${v}_${st}_$rep.json 2>/dev/null || exit $?
      python -c "
import json;d=json.loads(open('gpurun_out/r06v_${v}_${st}_$rep.json').read().strip().splitlines()[-1])
print('$v steps=$st rep=$rep', round(d['value']), round(d['ms_per_step']*1e3,2), round(d['kernel_ms']['persist_iteration']*1e3,2))"
    done
  done
done
