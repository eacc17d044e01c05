#!/bin/bash
# Instruction-mix PMC passes over a short MLP bench run (round 6: where a GEMM launch's fixed cost goes).
# usage: bash tools/pmc_insts.sh OUTDIR      (tools/pmc_insts_report.py reads the output)
out=$1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/$out
A="--steps 4 --warmup 2 --no-cpu-baseline --conv-steps 0 --ring-steps 0 --profile-rounds 1 --graph-rounds 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_MFMA --output-format csv -d $R/$out/i1 -- python3 $R/bench.py $A > $R/$out/i1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY --output-format csv -d $R/$out/i2 -- python3 $R/bench.py $A > $R/$out/i2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE SQ_INST_CYCLES_SALU --output-format csv -d $R/$out/i3 -- python3 $R/bench.py $A > $R/$out/i3.log 2>&1 || exit 1
