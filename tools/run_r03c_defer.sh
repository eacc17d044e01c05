# deferred head-loss reduction (CGL_HEAD_DEFER, default 1): the whole GPU suite, smoke(), then an interleaved
# A/B of the default bench line with CGL_HEAD_DEFER=1 / 0.  Each GPU step under its own limit.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c_defer
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gputest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
for v in 1 0 1 0 1 0; do
  CGL_HEAD_DEFER=$v timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 400 > $O/bench_$v.json 2> $O/bench_$v.err || exit $?
  python3 -c "import json; d=json.load(open('$O/bench_$v.json')); r=d['roofline']; p=d.get('parity',{}); print('DEFER=$v', d['ms_per_step'], r['per_kind_us_per_round'], p.get('pass'), p.get('d_loss_max_rel'), p.get('g_loss_max_rel'))" >> $O/summary.txt
done
