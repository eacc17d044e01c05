# round-3 diagnostics: launch-floor calibration, GEMM microbench, then the conv-round TA/TCP PMC
# pass of round 2 (which faulted) re-run once with serialized kernels so the fault names its kernel
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_diag
mkdir -p $O
timeout -k 10 60 $R/tools/latency_probe > $O/latency_probe.txt 2>&1 || exit $?
timeout -k 10 120 $R/tools/gemm_bench 200 > $O/gemm_bench.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
AMD_SERIALIZE_KERNEL=3 AMD_LOG_LEVEL=1 timeout -s KILL 150 rocprofv3 --pmc TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TOTAL_CACHE_ACCESSES --output-format csv -d $O/ta -- python3 $R/bench.py --model lsgan --steps 3 --warmup 1 --no-cpu-baseline --eager --profile-reps 1 > $O/ta.log 2>&1
echo "ta rc=$?" >> $O/ta.log
