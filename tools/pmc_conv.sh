#!/bin/bash
# Stall / instruction-mix PMC passes over a short conv (LSGAN) bench run: where the big conv kernels lose MFMA
# time.  usage: bash tools/pmc_conv.sh OUTDIR   (one counter group per rocprofv3 run; <= 8 SQ counters each)
out=$1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/$out
A="--model lsgan --steps 2 --warmup 1 --no-cpu-baseline"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $R/$out/c1 -- python3 $R/bench.py $A > $R/$out/c1.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $R/$out/c2 -- python3 $R/bench.py $A > $R/$out/c2.log 2>&1 || exit 1
