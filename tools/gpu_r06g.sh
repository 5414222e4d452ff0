#!/bin/bash
# Round 6: padded element-vector LDS rows of the chunk kernel (FEM_MF_FSPAD, default 1) -- matrix-free GPU tests, then
# tools/mf_probe.py A/B against the unpadded rows (build/var_fspad0), each twice, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_matfree.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r06g_tests.log 2>&1 || { tail -30 gpurun_out/r06g_tests.log; exit 1; }
tail -2 gpurun_out/r06g_tests.log
D=cuda-powered-mesh-handling-and-iterative-solvers_amd
for rep in 1 2; do
  for v in default fspad0; do
    L=$D/lib/libfem355.so; [ $v = fspad0 ] && L=$D/build/var_fspad0/libfem355.so
    FEM355_LIB=$L timeout -k 10 200 python tools/mf_probe.py --n 119 --no-assembled --iters 50 \
      > gpurun_out/r06g_mf_${v}_$rep.json 2>gpurun_out/r06g_mf_${v}_$rep.err || exit $?
    python -c "import json;d=json.load(open('gpurun_out/r06g_mf_${v}_$rep.json'));print('$v', round(d['k1_ms']*1e3,1), round(d['update_ms']*1e3,1), round(d['iter_ms']*1e3,1), round(d['it_per_s']))"
  done
done
