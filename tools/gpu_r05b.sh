#!/bin/bash
# Round-5 GPU pass B: the changed tests, the slot-position experiment (carried position with the prefetch records'
# fields defined vs left indeterminate), the element-chunk K1 timing, and a Poisson-only bench line (assembly time).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_matfree.py tests/test_dist_gpu.py tests/test_gpu_parity.py -m gpu \
    -k "matfree or fill_pass or scalar_mass or vals_edits or solver_layout or tile or refuses or concurrent or chunk" \
    > gpurun_out/pytest_b.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_b.log; [ $rc -ge 124 ] && exit $rc
for v in spcheck spundef; do
  V=cuda-powered-mesh-handling-and-iterative-solvers_amd/build/var_$v/libfem355.so
  FEM355_LIB=$PWD/$V timeout -k 10 300 python tools/mf_spcheck.py 40 60 80 119 > gpurun_out/$v.log 2>&1
  rc=$?; echo "== $v rc=$rc"; grep '^{' gpurun_out/$v.log; [ $rc -ge 124 ] && exit $rc
done
timeout -k 10 300 python tools/mf_probe.py --n 119 --iters 50 > gpurun_out/mf_probe_b.log 2>&1; rc=$?
tail -3 gpurun_out/mf_probe_b.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --elastic 0 \
    > gpurun_out/bench_b.log 2>&1; rc=$?; tail -c 1500 gpurun_out/bench_b.log; [ $rc -ne 0 ] && exit $rc
bash tools/mm_ab.sh
