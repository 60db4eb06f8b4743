# C4 train step kernel statistics, fp8 and bf16 (rocprofv3 --kernel-trace --stats)
# Usage (GPU box, repo root): bash tools/prof_c4.sh
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for p in fp8 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4_$p -o run -- python3 tools/c4_step.py $p 4 > gpurun_out/prof_c4_$p.log 2>&1
done
