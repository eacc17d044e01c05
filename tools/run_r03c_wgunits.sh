# conv round: weight-gradient wave units (CGL_WG_UNITS, pixel splits per tile) A/B, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c_wgunits
mkdir -p $O
for u in 2048 1024 1536 3072 2048; do
  CGL_WG_UNITS=$u timeout -k 10 300 python3 -u bench.py --model lsgan --no-cpu-baseline > $O/bench_$u.json 2> $O/bench_$u.err || exit $?
  python3 -c "import json; d=json.loads(open('$O/bench_$u.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$u', d['ms_per_step'], [(o['op'], o['geom'], o['us']) for o in r['ops'] if o['op']=='wgrad' and o['us']>50])" >> $O/summary.txt
done
