# instruction-cache / wait PMC pass of the default bench under two CGL_BN_FOLD settings
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_ic
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for f in 0 1; do
  CGL_BN_FOLD=$f timeout -s KILL 90 rocprofv3 --pmc SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAVES --output-format csv -d $O/ic$f -- python3 $R/bench.py --steps 3 --warmup 2 --profile-reps 1 --no-cpu-baseline > $O/ic$f.log 2>&1 || exit $?
done
