# round-3 (third session) check at HEAD after the container was re-created: the whole GPU suite, smoke(),
# the default bench line, the conv bench line, and rocprofv3 kernel stats of the MLP round.
# Each GPU step under its own limit; a time limit, abort or fault ends the script.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03c_head
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/gputest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 python3 -u bench.py --model lsgan --no-cpu-baseline > $O/bench_lsgan.json 2> $O/bench_lsgan.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || exit $?
echo done > $O/done.txt
