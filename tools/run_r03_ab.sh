# A/B of environment knobs on the default bench line: bash tools/run_r03_ab.sh OUT VAR "v1 v2 ..."
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for v in $3; do
  env $2=$v timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 300 > $O/bench_$v.json 2> $O/bench_$v.err || exit $?
  python3 -c "import json; d=json.load(open('$O/bench_$v.json')); r=d['roofline']; print('$2=$v', d['ms_per_step'], r['launches_per_round'], r['per_kind_us_per_round'], r['gemm_launch_us'])" >> $O/summary.txt
done
