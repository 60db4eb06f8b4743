#!/bin/bash
# Build a variant of libsmer_hip.so with extra compiler flags for A/B runs:
#   tools/build_variant.sh <name> -DFOO=1 ...   -> smer_music_generation_amd/_var/<name>.so
# VARIANT_ONLY="norm_embed.hip ..." applies the flags to those sources only.
# (load it with SMER_HIP_LIB=...; the in-tree library is untouched)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; shift
O=$R/smer_music_generation_amd/_var/$N
mkdir -p $O
for f in abi.cpp gemm.hip attention.hip norm_embed.hip train_ops.hip decode_ops.hip; do
  X=("$@")
  if [ -n "$VARIANT_ONLY" ] && [[ " $VARIANT_ONLY " != *" $f "* ]]; then X=(); fi
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -I$R/include -Xclang -target-feature -Xclang -packed-fp32-ops "${X[@]}" \
    -c $R/smer_music_generation_amd/csrc/$f -o $O/${f%.*}.o 2>/dev/null &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $O/*.o -o $R/smer_music_generation_amd/_var/$N.so
rm -rf $O
echo $R/smer_music_generation_amd/_var/$N.so
