#!/bin/bash
# Round 6: timing builds of the elastic value kernel (wrong values, no tests): pg = no gradients, pgs = no gradients
# and no column search, psw = no sweep, pall = none of the three -- the phase split of k_asm_tet4_acc<3>.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
KIND=elastic bash tools/asm_ab.sh pg pgs psw pall > gpurun_out/asm_s.log 2>&1 || exit $?
rm -rf gpurun_out/asmv_s; mv gpurun_out/asmv gpurun_out/asmv_s
for d in gpurun_out/asmv_s/*/; do echo "== $d"; python3 tools/kstats.py $d/run_kernel_stats.csv 3 | grep asm_tet4; done
