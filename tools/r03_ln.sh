#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "layernorm" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_ln_test.log 2>&1 &&
SMER_LN_BWD_T4=0 timeout -k 10 60 python tools/ln_bench.py > gpurun_out/r03_ln_bench.log 2>&1 &&
SMER_LN_BWD_T4=1 timeout -k 10 60 python tools/ln_bench.py >> gpurun_out/r03_ln_bench.log 2>&1 &&
timeout -k 10 300 python tools/ab_step.py c4 SMER_LN_BWD_T4 1 0 --rounds=1 > gpurun_out/r03_ab_ln.log 2>&1
