#!/bin/bash
# Build an experiment variant of libhecdna.so with extra compile definitions (development tool):
#   bash tools/variant_lib.sh <name> -DMACRO=value ...   -> tools/variants/<name>/libhecdna.so (HECDNA_LIB=...)
set -e
cd $(dirname $0)/..
NAME=$1; shift
PKG=homomorphic-encryption-algorithms-diploma-thesis_amd
OUT=tools/variants/$NAME
mkdir -p $OUT
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-function --offload-arch=gfx950 -Iinclude -I$PKG/csrc "$@" -c $PKG/csrc/hec_kernels.hip -o $OUT/hec_kernels.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $OUT/libhecdna.so $OUT/hec_kernels.o $PKG/build/hec_engine.o $PKG/build/hec_encode.o $PKG/build/hec_seal_io.o -ldl
rm -f $OUT/hec_kernels.o
echo $OUT/libhecdna.so
