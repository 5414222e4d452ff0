#!/bin/bash
# Chunk-kernel A/B: matrix-free GPU tests on the default build, then tools/mf_probe.py (10M elastic cube) for the
# default library and build/var_$1 (tools/build_variants.sh; $1 may list several, comma-separated), each twice,
# alternating. Output prefix: $2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VS=$(echo "$1" | tr ',' ' '); P=${2:-mfab}
[ -n "$SKIP_TESTS" ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_matfree.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${P}_tests.log 2>&1 || { tail -30 gpurun_out/${P}_tests.log; exit 1; }
tail -2 gpurun_out/${P}_tests.log
D=cuda-powered-mesh-handling-and-iterative-solvers_amd
for rep in 1 2; do
  for v in default $VS; do
    L=$D/lib/libfem355.so; [ $v != default ] && L=$D/build/var_$v/libfem355.so
    FEM355_LIB=$L timeout -k 10 200 python tools/mf_probe.py --n 119 --no-assembled --iters 50 \
      > gpurun_out/${P}_${v}_$rep.json 2>gpurun_out/${P}_${v}_$rep.err || exit $?
    python -c "import json;d=json.load(open('gpurun_out/${P}_${v}_$rep.json'));print('$v', round(d['k1_ms']*1e3,1), round(d['update_ms']*1e3,1), round(d['iter_ms']*1e3,1), round(d['it_per_s']))"
  done
done
