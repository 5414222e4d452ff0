#!/bin/bash
# Round 6 probes (2): the no-barrier timing probe of the persistent kernel (build/var_nobar) against the default build
# at 10M with the phase clock; rocprofv3 kernel stats of the world-1 RCCL element-partition line at the N = 8 rank
# share (n = 59) to split the matrix-free distributed iteration by kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in default nobar; do
  LIBV=cuda-powered-mesh-handling-and-iterative-solvers_amd/lib/libfem355.so
  [ $v = nobar ] && LIBV=cuda-powered-mesh-handling-and-iterative-solvers_amd/build/var_nobar/libfem355.so
  FEM355_LIB=$LIBV timeout -k 10 300 python tools/persist_check.py --n 119 --skip-solve --scheds 3 --prof --iters 300 \
    > gpurun_out/r06c_persist_$v.json 2>gpurun_out/r06c_persist_$v.err || exit $?
done
FEM355_PK_COOP=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r06c_prof_n59 -o run -- \
  python3 bench.py --force-dist --n 59 --steps 200 --warmup 20 --no-cpu-baseline --mixed 0 --reference-api 0 \
  > gpurun_out/r06c_dist_world1_n59.json 2>gpurun_out/r06c_dist_world1_n59.err || exit $?
find gpurun_out/r06c_prof_n59 -name "*kernel_stats.csv" | head -3
