set -o pipefail
mkdir -p gpurun_out/p7
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/p7/t.log 2>&1 &&
timeout -k 10 200 python3 tools/prof_infill.py > gpurun_out/p7/infill.log 2>&1 &&
timeout -k 10 300 python3 bench.py > gpurun_out/p7/bench.log 2>&1
rc=$?; tail -5 gpurun_out/p7/t.log; cat gpurun_out/p7/infill.log; tail -1 gpurun_out/p7/bench.log; exit $rc
