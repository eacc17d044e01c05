# kernel trace of the graph-replayed MLP round (one round's timeline per setting of $VAR)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_tl
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in ${VALS:-1}; do
  env ${VAR:-CGL_PACK}=$v CGL_PLAN_DEBUG=1 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tl$v -o run --output-format csv -- python3 -u $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --profile-reps 1 > $O/tl$v.log 2>&1 || exit $?
  python3 $R/tools/csv_round_timeline.py $(ls $O/tl$v/*kernel_trace.csv | head -1) cgl_round_prologue > $O/timeline$v.txt || exit $?
done
