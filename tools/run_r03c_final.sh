# round-3 closing evidence at HEAD: the whole GPU suite, smoke(), the default and conv bench lines, rocprofv3
# kernel stats of the MLP round, and the MLP FETCH_SIZE / WRITE_SIZE passes (one counter per run) for
# roofline.traffic.  Each GPU step under its own limit; a time limit, abort or fault ends the script.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03c_final
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gputest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 python3 -u bench.py --model lsgan --no-cpu-baseline > $O/bench_lsgan.json 2> $O/bench_lsgan.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $O/mlp_$c -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/mlp_$c.log 2>&1 || exit $?
done
echo done > $O/done.txt
