#!/bin/bash
# LDS bytes, vector and scalar registers of every kernel of the library (compiled device-only
# into a scratch directory): what decides how many blocks of a kernel fit on a CU beside the
# other streams' kernels.  tools/kernel_resources.sh [source.hip ...]
set -o pipefail
HERE=$(cd "$(dirname "$0")/.." && pwd)
SRC=$HERE/rempi_amd/csrc
TMP=$(mktemp -d)
LLVM=/opt/rocm/lib/llvm/bin
FILES=${@:-"encode lists chain chain_group chain_group8 decode"}
for f in $FILES; do
  f=$(basename $f .hip)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Xclang -target-feature -Xclang -packed-fp32-ops \
    --cuda-device-only -c $SRC/$f.hip -o $TMP/$f.co 2> >(grep -v "is not a recognized feature" >&2) || { echo "compile of $f failed"; exit 1; }
  $LLVM/clang-offload-bundler --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input=$TMP/$f.co --output=$TMP/$f.elf --unbundle
  $LLVM/llvm-readelf --notes $TMP/$f.elf | grep -E "^ +\.name:|group_segment_fixed_size|\.vgpr_count|\.sgpr_count|vgpr_spill_count" | paste - - - - - |
    awk '{ for (i = 1; i <= NF; i++) { if ($i == ".name:") n = $(i+1); if ($i == ".group_segment_fixed_size:") l = $(i+1); if ($i == ".vgpr_count:") v = $(i+1); if ($i == ".sgpr_count:") s = $(i+1); if ($i == ".vgpr_spill_count:") sp = $(i+1) } printf "%8d B LDS %4d VGPR %4d SGPR %3d spilled  %s\n", l, v, s, sp, n }' |
    while read -r line; do echo "$line" | sed -E 's/(_ZN4cdcx[0-9]+)(k_[a-z0-9_]+).*/\2/'; done
done | sort -k1,1nr
rm -rf $TMP
