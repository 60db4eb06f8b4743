#!/bin/bash
# the deferred-max attention test on the new and the previous library
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -q --timeout 120 --timeout-method thread"
V=$PWD/smer_music_generation_amd/_var
timeout -k 10 300 $T tests/test_kernels_gpu.py -k "attention" > gpurun_out/attn2_new.log 2>&1; r=$?
[ $r -le 1 ] || exit $r
SMER_HIP_LIB=$V/base.so timeout -k 10 300 $T tests/test_kernels_gpu.py -k "deferred" > gpurun_out/attn2_base.log 2>&1; r2=$?
grep -h "FAILED\|passed\|failed" gpurun_out/attn2_new.log gpurun_out/attn2_base.log
grep -h "AssertionError: assert" gpurun_out/attn2_new.log | head
exit $r
