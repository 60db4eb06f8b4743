#!/bin/bash
# Build a variant of libsmer_hip.so with extra -D flags for A/B timing:
#   tools/build_variant.sh <name> -DFOO=1 ...   -> smer_music_generation_amd/_var/<name>.so
# (load it with SMER_HIP_LIB=...; the in-tree library is untouched)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; shift
O=$R/smer_music_generation_amd/_var/$N
mkdir -p $O
for f in abi.cpp gemm.hip attention.hip norm_embed.hip train_ops.hip decode_ops.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -I$R/include "$@" \
    -c $R/smer_music_generation_amd/csrc/$f -o $O/${f%.*}.o &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $O/*.o -o $R/smer_music_generation_amd/_var/$N.so
rm -rf $O
echo $R/smer_music_generation_amd/_var/$N.so
