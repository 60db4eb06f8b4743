#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/bench_fp8_dgrad.py > gpurun_out/r03_f8iso2.log 2>&1 &&
timeout -k 10 300 python tools/ab_step.py c4 SMER_BWD_PRIO 0 1 --rounds=1 > gpurun_out/r03_ab_prio.log 2>&1 &&
timeout -k 10 300 python tools/ab_step.py c2 SMER_BWD_PRIO 0 1 >> gpurun_out/r03_ab_prio.log 2>&1
