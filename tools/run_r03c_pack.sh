# fragment-packed GEMM operands (CGL_PACK) at HEAD, after the latency cuts: interleaved A/B of the default line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c_pack
mkdir -p $O
for v in 1 0 1 0; do
  CGL_PACK=$v timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 400 > $O/bench_$v.json 2> $O/bench_$v.err || exit $?
  python3 -c "import json; d=json.load(open('$O/bench_$v.json')); r=d['roofline']; print('PACK=$v', d['ms_per_step'], r['per_kind_us_per_round'], d.get('parity',{}).get('pass'))" >> $O/summary.txt
done
