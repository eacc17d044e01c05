# vectorised round Adam (cgl_adam4) + bn_apply load hoist: the whole GPU suite, then an interleaved A/B of
# CGL_ADAM4=1 / 0 on the default bench line.  Each GPU step under its own limit.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c_adam4
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gputest.log; [ $rc -le 1 ] || exit $rc
for v in 1 0 1 0; do
  CGL_ADAM4=$v timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 400 > $O/bench_$v.json 2> $O/bench_$v.err || exit $?
  python3 -c "import json; d=json.load(open('$O/bench_$v.json')); r=d['roofline']; print('ADAM4=$v', d['ms_per_step'], r['per_kind_us_per_round'], d.get('parity',{}).get('pass'))" >> $O/summary.txt
done
