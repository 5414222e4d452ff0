#!/bin/bash
# assemble.hip variant with extra -D flags, linked with the other objects of the in-tree build (run make first):
# tools/build_asm_variant.sh NAME "-DFLAG=1 ..." -> .../build/var_NAME/libfem355.so (select with FEM355_LIB)
set -e
cd "$(dirname "$0")/../cuda-powered-mesh-handling-and-iterative-solvers_amd/csrc"
NAME=$1; FLAGS=$2
OUT=../build/var_$NAME
mkdir -p $OUT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -munsafe-fp-atomics $FLAGS -c assemble.hip -o $OUT/assemble.o
OBJS=$(ls ../build/*.o | grep -v assemble.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -Wl,-rpath,/opt/rocm/lib -L/opt/rocm/lib -lrccl $OBJS $OUT/assemble.o -o $OUT/libfem355.so
echo $OUT/libfem355.so
