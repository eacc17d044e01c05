# Round-3 closing evidence at HEAD: the whole GPU suite, smoke(), the bench lines of every model, rocprofv3
# kernel stats of the MLP round, the FETCH_SIZE / WRITE_SIZE traffic passes, and the prologue-fusion A/B.
# Every GPU step under its own limit; a time limit, abort or fault ends the script.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_ev
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gputest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py > $O/bench_mlp.json 2> $O/bench_mlp.err || exit $?
for m in lsgan mdgan mixg ring; do
  timeout -k 10 300 python3 -u bench.py --model $m --no-cpu-baseline > $O/bench_$m.json 2> $O/bench_$m.err || exit $?
done
for t in pro1 pro0 pro1b pro0b; do
  f=1; case $t in pro0*) f=0;; esac
  CGL_FUSE_PRO=$f timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 400 > $O/ab_$t.json 2> $O/ab_$t.err || exit $?
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $O/mlp_$c -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/mlp_$c.log 2>&1 || exit $?
done
echo done > $O/done.txt
