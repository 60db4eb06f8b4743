set -o pipefail
mkdir -p gpurun_out/p2
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -x -v --timeout 120 --timeout-method thread -k "grammar or generation or decode" > gpurun_out/p2/t.log 2>&1 &&
timeout -k 10 200 python3 tools/prof_infill.py > gpurun_out/p2/infill.log 2>&1
rc=$?; tail -15 gpurun_out/p2/t.log; cat gpurun_out/p2/infill.log; exit $rc
