#!/bin/bash
# Round 6 probes: (1) the no-barrier timing probe of the persistent kernel (build/var_nobar) against the default build
# at 10M with the phase clock; (2) world-1 RCCL element-partition lines at the N = 8 rank share (n = 59, 1.23M tets)
# and at 10M, both operators, for the configs[3] critical path.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
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
tail -c 300 gpurun_out/r06b_persist_nobar.json
