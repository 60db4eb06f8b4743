#!/bin/bash
# pipelined attention forward: attention GPU tests, kernel timings against
# the previous library (head.so), then C2 / C4 step A/B
set -o pipefail
mkdir -p gpurun_out
V=$PWD/smer_music_generation_amd/_var
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k attention > gpurun_out/a4_tests.log 2>&1
r=$?; tail -2 gpurun_out/a4_tests.log; [ $r -eq 0 ] || exit $r
for lib in head tree; do
  if [ $lib = tree ]; then L=""; else L="SMER_HIP_LIB=$V/$lib.so"; fi
  env $L timeout -k 10 200 python tools/bench_kernels.py attn > gpurun_out/a4_$lib.log 2>&1 || exit $?
  env $L timeout -k 10 300 python tools/bench_kernels.py attn_c4 >> gpurun_out/a4_$lib.log 2>&1 || exit $?
  echo "== $lib"; grep -v amdgpu.ids gpurun_out/a4_$lib.log
done
timeout -k 10 400 python tools/ab_step.py c2 SMER_HIP_LIB $V/head.so $PWD/smer_music_generation_amd/libsmer_hip.so --rounds=2 > gpurun_out/a4_c2.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/a4_c2.log | tail -2
timeout -k 10 500 python tools/ab_step.py c4 SMER_HIP_LIB $V/head.so $PWD/smer_music_generation_amd/libsmer_hip.so --rounds=2 > gpurun_out/a4_c4.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/a4_c4.log | tail -2
