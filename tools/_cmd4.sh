set -o pipefail
mkdir -p gpurun_out/p4
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread -k "decode or epilogue or generation or grammar or layouts" > gpurun_out/p4/t.log 2>&1 &&
timeout -k 10 120 python3 tools/bench_decode_kernels.py 32 1000 > gpurun_out/p4/dk.log 2>&1 &&
timeout -k 10 120 python3 tools/bench_decode_kernels.py 64 4096 >> gpurun_out/p4/dk.log 2>&1 &&
timeout -k 10 200 python3 tools/prof_infill.py > gpurun_out/p4/infill.log 2>&1
rc=$?; tail -5 gpurun_out/p4/t.log; cat gpurun_out/p4/dk.log gpurun_out/p4/infill.log; exit $rc
