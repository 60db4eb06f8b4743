#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/decode_ab.py 32 1000 SMER_DECODE_ODD_FIRST 1 0 > gpurun_out/r03_g.log 2>&1 &&
timeout -k 10 120 python tools/decode_ab.py 64 4096 SMER_DECODE_ODD_FIRST 1 0 >> gpurun_out/r03_g.log 2>&1
