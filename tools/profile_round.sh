#!/bin/bash
# Profile the headline bench: kernel-trace stats + separate PMC passes for
# FETCH_SIZE and WRITE_SIZE (never combined with other tracing domains),
# plus the decode step (graph replays), its HBM bytes (separate PMC passes),
# the C4 fp8 / bf16 train steps, SQ counters of the train step and of the
# fp8 vs bf16 forward GEMM.
# Usage (on the GPU box, from the repo root): bash tools/profile_round.sh <tag>
set -e
export TMPDIR=/tmp
R=$PWD
TAG=${1:-r01}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
# per-kernel durations in isolation: weight gradients on the main stream,
# as in bench.py's event-timed steps (the product path overlaps them)
export SMER_WGRAD_OVERLAP=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $R/bench.py --steps 5 --warmup 2 --no-infill --no-cpu --no-c4 > $OUT/trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- \
  python3 $R/bench.py --steps 2 --warmup 1 --no-infill --no-cpu --no-roofline --no-c4 > $OUT/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- \
  python3 $R/bench.py --steps 2 --warmup 1 --no-infill --no-cpu --no-roofline --no-c4 > $OUT/write.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/dec -o run -- \
  python3 $R/tools/prof_decode.py --n 50 --graph > $OUT/dec.log 2>&1
# the product path (weight-gradient stream overlap on), timed steps only
SMER_WGRAD_OVERLAP=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_ovl -o run -- \
  python3 $R/bench.py --steps 5 --warmup 2 --no-infill --no-cpu --no-c4 --no-roofline > $OUT/trace_ovl.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/dec_fetch -o run -- \
  python3 $R/tools/prof_decode.py --n 20 --graph > $OUT/dec_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/dec_write -o run -- \
  python3 $R/tools/prof_decode.py --n 20 --graph > $OUT/dec_write.log 2>&1
for p in fp8 bf16; do
  SMER_WGRAD_OVERLAP=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4_$p -o run -- \
    python3 $R/tools/c4_step.py $p 4 > $OUT/c4_$p.log 2>&1
done
# C4 fp8 with the weight gradients serialised: each kernel's own duration
SMER_WGRAD_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4ser -o run -- \
  python3 $R/tools/c4_step.py fp8 4 > $OUT/c4ser.log 2>&1
bash $R/tools/profile_pmc.sh $TAG > $OUT/pmc_sq.log 2>&1
bash $R/tools/pmc_fp8_gemm.sh > $OUT/pmc_fp8.log 2>&1
echo done
