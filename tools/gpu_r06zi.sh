#!/bin/bash
# Round 6 final: rocprofv3 kernel stats of the configs[4] mixed companion (stored-element-matrix assemblies after the
# repeated-node change) and of tools/mass_tile_probe.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export FEM355_PK_COOP=0
OUT=gpurun_out/prof_mixed
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 tools/mass_tile_probe.py --reps 5 > $OUT/trace.log 2>&1 || exit $?
find $OUT -name "*kernel_stats.csv" | head
echo zi-done
