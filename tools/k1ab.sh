cd "${GRAFT_REPO_ROOT}"
B=cuda-powered-mesh-handling-and-iterative-solvers_amd/build
for v in base u2 g1 nt0 base; do
  if [ $v = base ]; then unset FEM355_LIB; else export FEM355_LIB=$B/var_$v/libfem355.so; fi
  timeout -k 10 200 python bench.py --kind elastic --steps 200 --warmup 20 --no-cpu-baseline --dof-passes 1 > gpurun_out/k1_$v.log 2>&1 || exit $?
  tail -1 gpurun_out/k1_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['value']), d['kernel_ms'])"
done
