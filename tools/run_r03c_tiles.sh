# A/B of forced block shape + cross-workgroup split-K on the default bench line (env knobs only):
# each case "TILE/SPLITK"; "-/-" is the cost model's plan.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for c in -/- 1,1,4,2/4 1,1,4,2/2 1,1,4,1/2 1,1,4,2/0 -/-; do
  t=${c%/*}; k=${c#*/}; n=$(echo $c | tr ',/' '_-')
  ( [ "$t" != "-" ] && export CGL_GEMM_TILE=$t; [ "$k" != "-" ] && export CGL_SPLITK=$k;
    timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 300 > $O/bench_$n.json 2> $O/bench_$n.err ) || exit $?
  python3 -c "import json; d=json.load(open('$O/bench_$n.json')); r=d['roofline']; print('$c', d['ms_per_step'], r['per_kind_us_per_round'], r['gemm_launch_us'], d.get('parity',{}).get('pass'))" >> $O/summary.txt
done
