#!/bin/bash
# Round-5 GPU pass C: assembly A/B (solver layout formed in the SELL fill pass vs the separate pattern kernel) with
# kernel stats, then the rocprofv3 evidence for the bench line: kernel stats + FETCH_SIZE / WRITE_SIZE passes of the
# Poisson and elastic fixed-iteration runs, the element-chunk operator (tools/pmc_mf.sh), and FETCH/WRITE of the
# assembly kernels. Each --pmc pass is its own run; no trace domains beside --kernel-trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
KIND=poisson bash tools/asm_ab.sh env:FEM355_SL_SEPARATE=1 > gpurun_out/asm_ab_poisson.log 2>&1 || exit $?
mv gpurun_out/asmv gpurun_out/asmv_poisson
for f in gpurun_out/asmv_poisson/*.log; do echo "== $f"; grep '^{' $f | tail -2; done
KIND=elastic bash tools/asm_ab.sh > gpurun_out/asm_ab_elastic.log 2>&1 || exit $?
mv gpurun_out/asmv gpurun_out/asmv_elastic
tail -8 gpurun_out/asm_ab_elastic.log
BASE="--no-cpu-baseline --elastic 0 --mixed 0 --reference-api 0"
OUT=gpurun_out/prof_p PROF_ARGS="--steps 100 --warmup 10 $BASE" bash tools/profile_round.sh > /dev/null || exit $?
tail -1 gpurun_out/prof_p/trace.log
OUT=gpurun_out/prof_e PROF_ARGS="--kind elastic --steps 50 --warmup 5 --dof-passes 1 $BASE" bash tools/profile_round.sh > /dev/null || exit $?
tail -1 gpurun_out/prof_e/trace.log
OUT=gpurun_out/pmc_mf bash tools/pmc_mf.sh || exit $?
O=gpurun_out/pmc_asmfw
mkdir -p $O
for kind in poisson elastic; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -f csv -d $O/${kind}_$c -o run -- python3 tools/assemble_only.py --n 119 --kind $kind --reps 2 > $O/${kind}_$c.log 2>&1 || exit $?
  done
done
echo done
