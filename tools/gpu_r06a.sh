#!/bin/bash
# Round 6, first GPU pass: GPU tests + smoke + bench (tools/gpu_round.sh), then the no-barrier timing probe of the
# persistent kernel (build/var_nobar: wrong scalars, the neighbour-only coupling a pipelined iteration would leave)
# against the default build at 10M, each with the phase clock.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_round.sh all || exit $?
for v in default nobar; do
  LIBV=""; [ $v = nobar ] && LIBV=cuda-powered-mesh-handling-and-iterative-solvers_amd/build/var_nobar/libfem355.so
  FEM355_LIB=${LIBV:-cuda-powered-mesh-handling-and-iterative-solvers_amd/lib/libfem355.so} timeout -k 10 300 \
    python tools/persist_check.py --n 119 --skip-solve --scheds 3 --prof --iters 300 > gpurun_out/r06a_persist_$v.json 2>gpurun_out/r06a_persist_$v.err || exit $?
done
tail -c 600 gpurun_out/r06a_persist_default.json; echo; tail -c 600 gpurun_out/r06a_persist_nobar.json
