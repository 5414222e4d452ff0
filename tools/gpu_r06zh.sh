#!/bin/bash
# Round 6: k_graph's candidate loads issued G_KB = 4 passes at a time (default) vs one pass at a time (FEM_GRAPH_KB=1,
# build/var_kb1): pattern parity tests, then tools/pattern_only.py (c3d10 / c3d8 / c3d4) with each library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B=$PWD/cuda-powered-mesh-handling-and-iterative-solvers_amd/build
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "pattern or graph or hub or incidence or rcm or csr_abi or element_row_assembly" \
  > gpurun_out/r06zh_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r06zh_tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/r06zh_tests.log | head -20; exit $rc; }
for rep in 1 2; do
  for v in def kb1; do
    if [ $v = def ]; then unset FEM355_LIB; else export FEM355_LIB=$B/var_$v/libfem355.so; fi
    for f in c3d10 c3d8 c3d4; do
      echo "$v $f $(timeout -k 10 120 python tools/pattern_only.py --family $f --reps 7 2>/dev/null | tail -1)" || exit $?
    done
  done
done
echo zh-done
