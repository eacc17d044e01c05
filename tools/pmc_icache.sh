#!/bin/bash
# instruction-cache PMC pass over a short bench run (tools/pmc_report.py reads the output)
out=$1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/$out
timeout -s KILL 90 rocprofv3 --pmc SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQC_ICACHE_MISSES SQC_ICACHE_HITS --output-format csv -d $R/$out/ic -- python3 $R/bench.py --steps 3 --warmup 2 --profile-reps 1 --no-cpu-baseline > $R/$out/ic.log 2>&1
