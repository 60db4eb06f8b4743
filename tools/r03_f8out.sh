#!/bin/bash
# fp8 attention out-projections: kernel tests, attention timings, fp8
# training tests, C4 A/B of SMER_FP8_ATTN_OUT
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_kernels_gpu.py -k "attention" > gpurun_out/f8o_k.log 2>&1
r=$?; tail -2 gpurun_out/f8o_k.log; grep -h "^FAILED" gpurun_out/f8o_k.log | head; [ $r -eq 0 ] || exit $r
timeout -k 10 200 python tools/bench_kernels.py attn > gpurun_out/f8o_attn.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/f8o_attn.log
timeout -k 10 600 $T tests/test_prod_gpu.py > gpurun_out/f8o_prod.log 2>&1
r=$?; tail -2 gpurun_out/f8o_prod.log; grep -h "^FAILED\|C4 " gpurun_out/f8o_prod.log | head; [ $r -eq 0 ] || exit $r
timeout -k 10 600 python tools/ab_step.py c4 SMER_FP8_ATTN_OUT 0 1 --rounds=2 > gpurun_out/f8o_ab.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/f8o_ab.log | tail -2
