#!/bin/bash
# round-3 measurements: attention per shape (C2 + C4), grid-barrier cost, then the round's profile set
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/bench_kernels.py attn > gpurun_out/r03_attn.log 2>&1 &&
timeout -k 10 200 python tools/bench_kernels.py attn_c4 >> gpurun_out/r03_attn.log 2>&1 &&
timeout -k 10 60 tools/probes/gridbar_probe > gpurun_out/r03_gridbar.log 2>&1 &&
bash tools/profile_round.sh ${1:-r03a} > gpurun_out/r03_prof.log 2>&1
