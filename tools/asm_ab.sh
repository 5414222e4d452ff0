#!/bin/bash
# rocprofv3 kernel stats of the 10M elastic assembly: default build, then each variant named in $@
# (NAME = build/var_NAME/libfem355.so, or env:VAR=VAL for a runtime knob on the default build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
KIND=${KIND:-elastic}
mkdir -p gpurun_out/asmv
run() {  # name, then env assignments
  local name=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/asmv/$name -o run -- python3 tools/asm_breakdown.py --n 119 --kind $KIND --reps 5 > gpurun_out/asmv/$name.log 2>&1
}
run def FEM355_NONE=1 || exit $?
for v in "$@"; do
  case $v in
    env:*) kv=${v#env:}; run "${kv//=/_}" "$kv" || exit $? ;;
    *) run "$v" FEM355_LIB=cuda-powered-mesh-handling-and-iterative-solvers_amd/build/var_$v/libfem355.so || exit $? ;;
  esac
done
for d in gpurun_out/asmv/*/; do echo "== $d"; python3 tools/kstats.py $d/run_kernel_stats.csv 3; done
