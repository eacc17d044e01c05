# round-3 evidence: the whole GPU suite, smoke(), then (last: it faulted once in round 2) the conv
# round's TA/TCP PMC pass of round 2, unserialized, exactly as tools/pmc_passes.sh ran it
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_suite
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/gputest.log
[ $rc -le 1 ] || exit $rc          # a time limit, abort or fault: nothing more on the GPU
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
if [ -n "$TA" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 150 rocprofv3 --pmc TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TOTAL_CACHE_ACCESSES --output-format csv -d $O/ta -- python3 $R/bench.py --model lsgan --steps 3 --warmup 1 --no-cpu-baseline --eager --profile-reps 1 > $O/ta.log 2>&1
  echo "ta rc=$?" >> $O/ta.log
fi
