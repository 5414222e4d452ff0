cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/asm
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/asm/p -o run -- python3 tools/asm_breakdown.py --n 119 --kind poisson --reps 5 > gpurun_out/asm/p.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/asm/e -o run -- python3 tools/asm_breakdown.py --n 119 --kind elastic --reps 5 > gpurun_out/asm/e.log 2>&1
