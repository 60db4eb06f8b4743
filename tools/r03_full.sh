#!/bin/bash
# round-3 full check on the GPU box: the -m gpu suite, smoke(), the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r03_gputest.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/r03_bench.log 2>&1
