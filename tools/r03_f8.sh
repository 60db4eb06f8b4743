#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_prod_gpu.py tests/test_kernels_gpu.py -k "fp8 or layernorm" -v --timeout 200 --timeout-method thread > gpurun_out/r03_f8_test.log 2>&1 &&
timeout -k 10 400 python tools/ab_step.py c4 SMER_FP8_DGRAD 1 0 --rounds=1 > gpurun_out/r03_ab_f8.log 2>&1
