#!/bin/bash
# Round-5 GPU pass H: gather windows from per-slice spans (no atomics) -- solver-layout / persistent-schedule parity,
# the Poisson assembly timeline, and the Poisson bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_parity.py tests/test_gpu_dist_persist.py -m gpu \
    -k "solver_layout or fill_pass or uniform or tile or persist or window" > gpurun_out/pytest_h.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_h.log; [ $rc -ne 0 ] && exit $rc
KIND=poisson bash tools/asm_ab.sh > gpurun_out/asm_h.log 2>&1 || exit $?
rm -rf gpurun_out/asmv_h; mv gpurun_out/asmv gpurun_out/asmv_h
python3 tools/kstats.py gpurun_out/asmv_h/def/run_kernel_stats.csv 8; grep '^{' gpurun_out/asmv_h/def.log | head -c 300; echo
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --elastic 0 --mixed 0 \
    > gpurun_out/bench_h.log 2>&1; rc=$?; tail -c 1200 gpurun_out/bench_h.log; exit $rc
