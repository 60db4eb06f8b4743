#!/bin/bash
# round-3 GEMM calibration: smer vs hipBLASLt per shape, per-shape time in the C2 step
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 180 python tools/blas_calib.py > gpurun_out/r03_blas.log 2>&1 &&
timeout -k 10 180 python tools/bench_wgrad.py > gpurun_out/r03_wgrad.log 2>&1 &&
timeout -k 10 240 python tools/gemm_shapes.py bf16 > gpurun_out/r03_shapes.log 2>&1
