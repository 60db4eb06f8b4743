set -o pipefail
mkdir -p gpurun_out/p5
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread -k "decode or generation or grammar" > gpurun_out/p5/t.log 2>&1 &&
timeout -k 10 200 python3 tools/prof_infill.py > gpurun_out/p5/infill.log 2>&1
rc=$?; tail -25 gpurun_out/p5/t.log; cat gpurun_out/p5/infill.log; exit $rc
