#!/bin/bash
# full -m gpu suite + bench after the round-3 changes, then a GEMM64 A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r03_gputest2.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/r03_bench2.log 2>&1 &&
timeout -k 10 300 python tools/ab_step.py c2 SMER_GEMM64 1 0 > gpurun_out/r03_ab_g64.log 2>&1
