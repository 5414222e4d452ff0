#!/bin/bash
# Round-5 GPU pass: GPU tests + smoke, the slot-position debug probe (FEM_MF_SPCHECK build), the N>1 path at world
# size 1 (RCCL element partition incl. the matrix-free operator: bench.py --force-dist), then the default bench line.
# Each step has its own limit; a fault stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then bash tools/gpu_round.sh tests || exit $?; fi
V=cuda-powered-mesh-handling-and-iterative-solvers_amd/build/var_spcheck/libfem355.so
if [ -f $V ]; then
  FEM355_LIB=$PWD/$V timeout -k 10 300 python tools/mf_spcheck.py 20 40 60 80 119 > gpurun_out/spcheck.log 2>&1
  rc=$?; cat gpurun_out/spcheck.log | grep '^{'; [ $rc -ge 124 ] && exit $rc
fi
timeout -k 10 600 python bench.py --force-dist --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
    > gpurun_out/bench_dist1.log 2>&1 || { echo "dist1 rc=$?"; tail -30 gpurun_out/bench_dist1.log; exit 1; }
tail -c 3000 gpurun_out/bench_dist1.log
BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu_round.sh bench
