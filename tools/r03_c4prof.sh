#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c4ser
SMER_WGRAD_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4ser -o run -- python3 tools/c4_step.py fp8 4 > gpurun_out/c4ser/log 2>&1 &&
timeout -k 10 300 python tools/gemm_shapes.py fp8 c4 > gpurun_out/r03_c4_shapes.log 2>&1
