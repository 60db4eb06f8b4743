#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_prod_gpu.py -k "gemm_epilogue or gemm_layouts or greedy or sampled or batch_matches or warm_session or c5_fp32" -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_e_test.log 2>&1 &&
timeout -k 10 120 python tools/capture_probe.py > gpurun_out/r03_e_capture.log 2>&1 &&
timeout -k 10 200 python bench.py --no-c4 --no-c5 --no-cpu > gpurun_out/r03_e_bench.log 2>&1
