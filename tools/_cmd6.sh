set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/p6
timeout -k 10 120 python3 tools/bench_decode_kernels.py 32 1000 > gpurun_out/p6/dk.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p6/dec -o run -- python3 tools/prof_decode.py --n 50 --graph > gpurun_out/p6/dec.log 2>&1
rc=$?; cat gpurun_out/p6/dk.log gpurun_out/p6/dec.log; exit $rc
