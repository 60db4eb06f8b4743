#!/bin/bash
# ring GEMM: parity test, isolated shapes, C2 bench A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "ring or gemm256 or gemm_layouts or gemm_epilogue" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_ring_test.log 2>&1 &&
SMER_GEMM_RING=1 timeout -k 10 120 python tools/blas_calib.py > gpurun_out/r03_ring_blas1.log 2>&1 &&
SMER_GEMM_RING=0 timeout -k 10 120 python tools/blas_calib.py > gpurun_out/r03_ring_blas0.log 2>&1 &&
SMER_GEMM_RING=1 timeout -k 10 200 python bench.py --no-infill --no-cpu --no-c4 --steps 20 --warmup 5 > gpurun_out/r03_ring_bench1.log 2>&1 &&
SMER_GEMM_RING=0 timeout -k 10 200 python bench.py --no-infill --no-cpu --no-c4 --steps 20 --warmup 5 > gpurun_out/r03_ring_bench0.log 2>&1
