#!/bin/bash
# Round 6: the gather-free distributed element-chunk iteration (FEM_MF_DIST_NOGATHER, build/var_nogather) against the
# default: distributed GPU tests on the variant, then world-1 RCCL lines at the N = 8 rank share and at 10M for both,
# and rocprofv3 kernel stats of both at the rank share.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
D=cuda-powered-mesh-handling-and-iterative-solvers_amd
FEM355_LIB=$D/build/var_nogather/libfem355.so timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06n_tests.log 2>&1 || { tail -30 gpurun_out/r06n_tests.log; exit 1; }
tail -2 gpurun_out/r06n_tests.log
for v in default nogather; do
  L=$D/lib/libfem355.so; [ $v = nogather ] && L=$D/build/var_nogather/libfem355.so
  for n in 59 119; do
    FEM355_LIB=$L timeout -k 10 400 python bench.py --force-dist --n $n --steps 200 --warmup 20 --no-cpu-baseline \
      --mixed 0 --reference-api 0 > gpurun_out/r06n_${v}_n$n.json 2>gpurun_out/r06n_${v}_n$n.err || exit $?
    python -c "
import json;d=json.loads(open('gpurun_out/r06n_${v}_n$n.json').read().strip().splitlines()[-1]);m=d['elasticity']['element_rccl']['matfree']
print('$v n$n', round(m['ms_per_step']*1e3,2), {a: round(b*1e3,2) for a,b in m['kernel_ms'].items()}, m['solve_iters'])"
  done
  FEM355_LIB=$L FEM355_PK_COOP=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06n_prof_$v -o run -- \
    python3 bench.py --force-dist --n 59 --steps 200 --warmup 20 --no-cpu-baseline --mixed 0 --reference-api 0 \
    > gpurun_out/r06n_prof_$v.log 2>&1 || exit $?
done
