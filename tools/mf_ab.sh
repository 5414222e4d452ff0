#!/bin/bash
# A/B of element-chunk operator builds (run on the GPU box): tools/mf_probe.py with the default library and with each
# variant library named (cuda-powered-mesh-handling-and-iterative-solvers_amd/build/var_NAME/libfem355.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/mf_ab}
mkdir -p $O
ARGS=${MF_ARGS:-"--n 119 --no-assembled --iters 50"}
timeout -k 10 150 python3 tools/mf_probe.py $ARGS > $O/default.log 2>&1 || exit $?
echo "default $(tail -1 $O/default.log)"
for v in "$@"; do   # a variant library name, or NAME=VALUE: the default library with that environment variable
  if [[ "$v" == *=* ]]; then
    env "$v" timeout -k 10 150 python3 tools/mf_probe.py $ARGS > $O/env_$v.log 2>&1 || exit $?
    echo "$v $(tail -1 $O/env_$v.log)"
  else
    FEM355_LIB=cuda-powered-mesh-handling-and-iterative-solvers_amd/build/var_$v/libfem355.so timeout -k 10 150 python3 tools/mf_probe.py $ARGS > $O/$v.log 2>&1 || exit $?
    echo "$v $(tail -1 $O/$v.log)"
  fi
done
