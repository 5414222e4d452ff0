#!/bin/bash
# Builds libfem355.so variants with extra -D flags for A/B probes: tools/build_variants.sh NAME "-DFLAG=1 ..."
# -> cuda-powered-mesh-handling-and-iterative-solvers_amd/build/var_NAME/libfem355.so (select with FEM355_LIB)
set -e
cd "$(dirname "$0")/../cuda-powered-mesh-handling-and-iterative-solvers_amd/csrc"
NAME=$1; FLAGS=$2
OUT=../build/var_$NAME
mkdir -p $OUT
OBJS=""
for f in runtime pattern assemble pcg stress topology csr_abi reorder matfree; do
  EX=""; [ $f = pcg ] && EX="-mllvm -disable-promote-alloca-to-vector"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -munsafe-fp-atomics $EX $FLAGS -c $f.hip -o $OUT/$f.o &
  OBJS="$OBJS $OUT/$f.o"
done
g++ -O2 -std=c++17 -fPIC -Wall -c vtk.cpp -o $OUT/vtk.o
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -Wl,-rpath,/opt/rocm/lib -L/opt/rocm/lib -lrccl $OBJS $OUT/vtk.o -o $OUT/libfem355.so
echo $OUT/libfem355.so
