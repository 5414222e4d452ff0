#!/bin/bash
# one source's variant (SRC=assemble by default, or pattern, pcg, ...) with extra -D flags, linked with the other
# objects of the in-tree build (run make first):
# [SRC=pattern] tools/build_asm_variant.sh NAME "-DFLAG=1 ..." -> .../build/var_NAME/libfem355.so (FEM355_LIB)
set -e
cd "$(dirname "$0")/../cuda-powered-mesh-handling-and-iterative-solvers_amd/csrc"
NAME=$1; FLAGS=$2
OUT=../build/var_$NAME
mkdir -p $OUT
SRC=${SRC:-assemble}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -munsafe-fp-atomics $FLAGS -c $SRC.hip -o $OUT/$SRC.o
OBJS=$(ls ../build/*.o | grep -v "/$SRC.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -Wl,-rpath,/opt/rocm/lib -L/opt/rocm/lib -lrccl $OBJS $OUT/$SRC.o -o $OUT/libfem355.so
echo $OUT/libfem355.so
