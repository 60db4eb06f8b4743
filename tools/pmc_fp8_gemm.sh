#!/bin/bash
# fp8 vs bf16 forward GEMM counters (one shape, M65536 N2304 K3072): MFMA busy,
# LDS bank conflicts, waits (tools/pmc_sq.py), kernel durations.
# Usage (GPU box, repo root): bash tools/pmc_fp8_gemm.sh
set -e
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/pmc_fp8
mkdir -p $OUT
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for k in fp8 fwd; do
  timeout -s KILL 60 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d $OUT/$k -o run -- python3 $R/tools/gemm_one_shape.py $k 65536 2304 3072 10 > $OUT/$k.log 2>&1
done
python3 $R/tools/pmc_sq.py $OUT/sq.json $(find $OUT -name '*counter_collection.csv') > $OUT/sq.txt
timeout -k 10 60 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 $R/tools/gemm_one_shape.py fp8 65536 2304 3072 10 > $OUT/kt.log 2>&1
echo done
