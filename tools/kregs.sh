#!/bin/bash
# VGPR / spill / LDS per kernel of the built engine object (development tool)
# usage: bash tools/kregs.sh [regex]
set -e
O=${KO:-$(dirname $0)/../homomorphic-encryption-algorithms-diploma-thesis_amd/build/hec_kernels.o}
T=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$T/fat.bin $O
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$T/fat.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/k.co
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $T/k.co | grep -E "^\s+\.(name|vgpr_count|vgpr_spill_count|group_segment_fixed_size|private_segment_fixed_size|sgpr_spill_count):" | paste - - - - - - | sed 's/  */ /g' | grep -E "${1:-.}"
rm -rf $T
