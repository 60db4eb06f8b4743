#!/bin/bash
# forward without in-loop spills: attention tests + per-shape timings, C4 A/B
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_kernels_gpu.py -k "attention" > gpurun_out/f8o2_k.log 2>&1
r=$?; tail -1 gpurun_out/f8o2_k.log; grep -h "^FAILED" gpurun_out/f8o2_k.log | head; [ $r -eq 0 ] || exit $r
timeout -k 10 200 python tools/bench_kernels.py attn > gpurun_out/f8o2_attn.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_kernels.py attn_c4 >> gpurun_out/f8o2_attn.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/f8o2_attn.log
timeout -k 10 600 python tools/ab_step.py c4 SMER_FP8_ATTN_OUT 0 1 --rounds=2 > gpurun_out/f8o2_ab.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/f8o2_ab.log | tail -2
