# after the descriptor-upload fix: the new upload-order / short-batch / canary GPU tests, then the
# conv round's TA/TCP PMC pass exactly as tools/run_r03_suite.sh ran it (it faulted there), then the
# FETCH_SIZE / WRITE_SIZE traffic passes (tools/run_r03_traffic.sh)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_fix
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_upload_order.py tests/test_gpu_short_batch.py tests/test_gpu_conv_stats_canary.py -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TOTAL_CACHE_ACCESSES --output-format csv -d $O/ta -- python3 $R/bench.py --model lsgan --steps 3 --warmup 1 --no-cpu-baseline --eager --profile-reps 1 > $O/ta.log 2>&1
rc=$?
echo "ta rc=$rc" >> $O/ta.log
[ $rc -eq 0 ] || exit $rc
bash $R/tools/run_r03_traffic.sh
