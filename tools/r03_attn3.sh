#!/bin/bash
# attention kernel timings: previous commit (head.so), the in-tree library,
# and the -fno-slp-vectorize variant; then the attention tests in-tree
set -o pipefail
mkdir -p gpurun_out
V=$PWD/smer_music_generation_amd/_var
for lib in head tree noslp; do
  if [ $lib = tree ]; then L=""; else L="SMER_HIP_LIB=$V/$lib.so"; fi
  env $L timeout -k 10 200 python tools/bench_kernels.py attn > gpurun_out/a3_$lib.log 2>&1 || exit $?
  env $L timeout -k 10 300 python tools/bench_kernels.py attn_c4 >> gpurun_out/a3_$lib.log 2>&1 || exit $?
done
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k attention > gpurun_out/a3_tests.log 2>&1
r=$?
for lib in head tree noslp; do echo "== $lib"; grep -v amdgpu.ids gpurun_out/a3_$lib.log; done
tail -2 gpurun_out/a3_tests.log
exit $r
