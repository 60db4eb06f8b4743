set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/p1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p1/train -o run -- python3 bench.py --steps 5 --warmup 2 --no-infill --no-cpu > gpurun_out/p1/train.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p1/dec -o run -- python3 tools/prof_decode.py --n 50 > gpurun_out/p1/dec.log 2>&1 &&
timeout -k 10 200 python3 tools/prof_infill.py > gpurun_out/p1/infill.log 2>&1 &&
timeout -k 10 200 python3 tools/bench_kernels.py all > gpurun_out/p1/kern.log 2>&1
echo rc=$?
