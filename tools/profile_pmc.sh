#!/bin/bash
# SQ / GRBM counter passes over the C2 train step (weight gradients on the
# main stream so each kernel's counters are its own): MFMA busy, LDS bank
# conflicts, wait breakdown, instruction mix.  One rocprofv3 run per pass
# (never combined with tracing domains), each under its own kill timeout.
# Usage (GPU box, repo root): bash tools/profile_pmc.sh <tag>
set -e
export TMPDIR=/tmp
R=$PWD
TAG=${1:-r02}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
export SMER_WGRAD_OVERLAP=0
B="python3 $R/bench.py --steps 2 --warmup 1 --no-infill --no-cpu --no-roofline --no-c4"
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU_MFMA_BF16 SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $P1 --output-format csv -d $OUT/p1 -o run -- $B > $OUT/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc $P2 --output-format csv -d $OUT/p2 -o run -- $B > $OUT/p2.log 2>&1
python3 $R/tools/pmc_sq.py $OUT/sq.json $(find $OUT/p1 -name '*counter_collection.csv') $(find $OUT/p2 -name '*counter_collection.csv') > $OUT/sq.txt
echo done
