#!/bin/bash
# attention: GPU tests (new library + variants), the deferred-max test on the
# previous library (a check of the test itself), kernel timings per library.
# Test failures (rc 1) do not stop the script; anything else does.
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -q --timeout 120 --timeout-method thread"
V=$PWD/smer_music_generation_amd/_var
ok() { [ $1 -le 1 ]; }
for lib in new base lsum; do
  if [ $lib = new ]; then L=""; else L="SMER_HIP_LIB=$V/$lib.so"; fi
  env $L timeout -k 10 400 $T tests/test_kernels_gpu.py -k "attention" > gpurun_out/attn_tests_$lib.log 2>&1
  r=$?; echo "rc $r" >> gpurun_out/attn_tests_$lib.log; ok $r || exit $r
done
for lib in new base lsum; do
  if [ $lib = new ]; then L=""; else L="SMER_HIP_LIB=$V/$lib.so"; fi
  env $L timeout -k 10 200 python tools/bench_kernels.py attn > gpurun_out/attn_$lib.log 2>&1 || exit $?
  env $L timeout -k 10 300 python tools/bench_kernels.py attn_c4 > gpurun_out/attn_c4_$lib.log 2>&1 || exit $?
done
for lib in new base lsum; do echo "== $lib"; tail -2 gpurun_out/attn_tests_$lib.log; grep FAILED gpurun_out/attn_tests_$lib.log | head; cat gpurun_out/attn_$lib.log gpurun_out/attn_c4_$lib.log; done
