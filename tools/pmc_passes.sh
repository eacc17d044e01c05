#!/bin/bash
# PMC passes over a short bench run (one counter group per rocprofv3 run, MI355X_MICROARCH.md limits).
# usage: bash tools/pmc_passes.sh OUTDIR [bench args...]
out=$1; shift
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
run() {
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $R/$out/$1 -- python3 $R/bench.py $BENCH_ARGS > $R/$out/$1.log 2>&1
}
mkdir -p $R/$out
run SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM || exit 1
run TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TOTAL_CACHE_ACCESSES || exit 1
run SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU || exit 1
if [ -n "$PMC_TRAFFIC" ]; then
  run FETCH_SIZE || exit 1
  run WRITE_SIZE || exit 1
fi
