#!/bin/bash
# Round 6 probes: matrix-free GPU tests (the dof-pair merged update), the single-GPU bench line (Poisson + elasticity
# + element-chunk operator), the no-barrier timing probe of the persistent kernel (build/var_nobar) against the
# default build at 10M with the phase clock, then world-1 RCCL element-partition lines at the N = 8 rank share (n = 59,
# 1.23M tets) and at 10M, both operators (configs[3] critical path).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_matfree.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r06b_matfree_tests.log 2>&1 || { tail -20 gpurun_out/r06b_matfree_tests.log; exit 1; }
tail -2 gpurun_out/r06b_matfree_tests.log
timeout -k 10 400 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --mixed 0 --reference-api 0 \
  > gpurun_out/r06b_bench.json 2>gpurun_out/r06b_bench.err || exit $?
for v in default nobar; do
  LIBV=cuda-powered-mesh-handling-and-iterative-solvers_amd/lib/libfem355.so
  [ $v = nobar ] && LIBV=cuda-powered-mesh-handling-and-iterative-solvers_amd/build/var_nobar/libfem355.so
  FEM355_LIB=$LIBV timeout -k 10 300 python tools/persist_check.py --n 119 --skip-solve --scheds 3 --prof --iters 300 \
    > gpurun_out/r06b_persist_$v.json 2>gpurun_out/r06b_persist_$v.err || exit $?
done
for n in 59 119; do
  timeout -k 10 400 python bench.py --force-dist --n $n --steps 200 --warmup 20 --no-cpu-baseline --mixed 0 \
    --reference-api 0 > gpurun_out/r06b_dist_world1_n$n.json 2>gpurun_out/r06b_dist_world1_n$n.err || exit $?
done
