#!/bin/bash
# Round-5 GPU pass I: tail prefetches clamped to the workgroup's last chunk (matrix-free parity + K1 traffic), the
# pattern sizes in one launch (pattern parity + Poisson assembly timeline).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_matfree.py tests/test_dist_gpu.py tests/test_gpu_parity.py -m gpu \
    -k "matfree or chunk or mf or pattern or graph or solver_layout or fill_pass or persist or coalesce" \
    > gpurun_out/pytest_i.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_i.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/mf_probe.py --n 119 --no-assembled --iters 50 > gpurun_out/mfprof_i.log 2>&1 || exit $?
grep '^{' gpurun_out/mfprof_i.log | tail -1 | head -c 600; echo
O=gpurun_out/pmc_mf_i; mkdir -p $O
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $c -f csv -d $O/${c} -o run -- python3 tools/mf_probe.py --n 119 --no-assembled --iters 10 > $O/$c.log 2>&1 || exit $?
done
KIND=poisson bash tools/asm_ab.sh > gpurun_out/asm_i.log 2>&1 || exit $?
rm -rf gpurun_out/asmv_i; mv gpurun_out/asmv gpurun_out/asmv_i; grep '^{' gpurun_out/asmv_i/def.log | head -c 300; echo
