set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-infill --no-cpu --no-roofline > gpurun_out/b_c4.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o run -- python3 tools/c4_step.py fp8 > gpurun_out/prof_c4.log 2>&1
