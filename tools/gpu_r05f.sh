#!/bin/bash
# Round-5 GPU pass F: solver-layout parity after the 32-bit pair stores; the fused fill pass with parts of the solver
# layout skipped (FEM_SL_SKIP timing builds); counters of the element-chunk K1 after the rotated prefetch records.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_parity.py -m gpu -k "solver_layout or fill_pass or uniform or tile or persist" \
    > gpurun_out/pytest_f.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_f.log; [ $rc -ne 0 ] && exit $rc
KIND=poisson bash tools/asm_ab.sh slskip1 slskip2 slskip4 > gpurun_out/asm_f.log 2>&1 || exit $?
rm -rf gpurun_out/asmv_f; mv gpurun_out/asmv gpurun_out/asmv_f
for d in gpurun_out/asmv_f/*/; do echo "== $d"; python3 tools/kstats.py $d/run_kernel_stats.csv 3 | grep -E "fill_graph|asm_tet4"; done
O=gpurun_out/pmc_mf_f
ARGS="--n 119 --no-assembled --iters 10"
C2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAIT_INST_LDS"
C3="TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum"
OUT=$O bash tools/pmc_mf.sh || exit $?
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $C2 -f csv -d $O/c2 -o run -- python3 tools/mf_probe.py $ARGS > $O/c2.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $C3 -f csv -d $O/c3 -o run -- python3 tools/mf_probe.py $ARGS > $O/c3.log 2>&1 || exit $?
echo done
