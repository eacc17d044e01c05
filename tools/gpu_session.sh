#!/bin/bash
# One GPU-box session of named steps, each under its own time limit; a failing step ends the session.
#   bash tools/gpu_session.sh TAG step [step ...]        (outputs under gpurun_out/TAG/)
# steps:
#   tests        the whole pytest -m gpu suite                      -> gputest.log
#   tests:FILES  a subset (comma-separated test files)              -> gputest.log
#   smoke        __graft_entry__.smoke()                            -> smoke.log
#   bench        bench.py default line (N = 1, with CPU baseline)   -> bench.json
#   bench:ARGS   bench.py with ARGS (commas become spaces)          -> bench_<n>.json
#   lsgan        bench.py --model lsgan --no-cpu-baseline           -> bench_lsgan.json
#   prof         rocprofv3 --kernel-trace --stats of a short MLP bench -> prof/ (kernel_stats.csv)
#   proflsgan    the same for the conv round                        -> prof_lsgan/
#   traffic      FETCH_SIZE and WRITE_SIZE passes (one counter per run) of the MLP bench -> mlp_FETCH_SIZE/ ...
#   trafficlsgan the same two passes of the conv round (LSGAN bench)      -> lsgan_FETCH_SIZE/ ...
#   tiles[:ARGS] tools/tile_search.py (in-round per-descriptor tile search) -> tile_search.json / .log
#   ab:T1=ENV1;T2=ENV2   the MLP bench under env settings, interleaved x3 -> ab_<T>_<i>.json
#   abl:T1=ENV1;T2=ENV2  the same for the LSGAN conv round, interleaved x2 -> abl_<T>_<i>.json
#   capprobe     tools/capture_probe.py, every case (torch.cuda.graph capture cases, one subprocess each) -> capture_probe.txt
#   rccl         the RCCL world-1 worker with the split-round timing -> rccl.log
#   gemmtrace[:TAG]  per-workgroup GEMM phase stamps in the graph round (lib_TAG, default lib_trace) -> gemm_trace_TAG.json
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
n=0
for st in "$@"; do
  n=$((n + 1))
  name=${st%%:*}; arg=""; [ "$name" != "$st" ] && arg=${st#*:}
  echo "[$(date +%T)] step $n: $st" | tee -a $O/session.log
  case $name in
    tests)
      files=tests; [ -n "$arg" ] && files=${arg//,/ }
      timeout -k 10 1200 python3 -u -m pytest $files -m gpu -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
      rc=$?; echo "pytest rc=$rc" >> $O/gputest.log; tail -3 $O/gputest.log; [ $rc -le 1 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $? ;;
    bench)
      if [ -n "$arg" ]; then
        timeout -k 10 400 python3 -u bench.py ${arg//,/ } > $O/bench_$n.json 2> $O/bench_$n.err || exit $?
      else
        timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
      fi ;;
    lsgan)
      timeout -k 10 400 python3 -u bench.py --model lsgan --no-cpu-baseline > $O/bench_lsgan.json 2> $O/bench_lsgan.err || exit $? ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
        python3 $R/bench.py --steps 50 --warmup 10 --no-cpu-baseline --conv-steps 0 --ring-steps 0 > $O/prof.log 2>&1) || exit $? ;;
    proflsgan)
      # proflsgan:TAG=ENV1,ENV2 profiles under those env settings -> prof_lsgan_TAG/
      d=prof_lsgan; envs=""
      if [ -n "$arg" ]; then d=prof_lsgan_${arg%%=*}; envs=${arg#*=}; envs=${envs//,/ }; fi
      (cd /tmp && export TMPDIR=/tmp $envs && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$d -o run -- \
        python3 $R/bench.py --model lsgan --steps 10 --warmup 3 --no-cpu-baseline > $O/$d.log 2>&1) || exit $? ;;
    traffic)
      for c in FETCH_SIZE WRITE_SIZE; do
        (cd /tmp && export TMPDIR=/tmp CGL_PLAN_DEBUG=1 && timeout -s KILL 150 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/mlp_$c -o run -- \
          python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --conv-steps 0 --ring-steps 0 > $O/mlp_$c.log 2>&1) || exit $?
      done ;;
    trafficlsgan)
      for c in FETCH_SIZE WRITE_SIZE; do
        (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 200 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/lsgan_$c -o run -- \
          python3 $R/bench.py --model lsgan --steps 4 --warmup 2 --no-cpu-baseline > $O/lsgan_$c.log 2>&1) || exit $?
      done ;;
    tiles)
      timeout -k 10 600 python3 -u tools/tile_search.py ${arg//,/ } --out $O/tile_search.json > $O/tile_search.log 2>&1 || exit $? ;;
    ab)
      IFS=';' read -ra pairs <<< "$arg"
      for i in 1 2 3; do
        for kv in "${pairs[@]}"; do
          t=${kv%%=*}; envs=${kv#*=}
          env $envs timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --conv-steps 0 --steps 400 > $O/ab_${t}_$i.json 2> $O/ab_${t}_$i.err || exit $?
        done
      done ;;
    abl)
      IFS=';' read -ra pairs <<< "$arg"
      for i in 1 2; do
        for kv in "${pairs[@]}"; do
          t=${kv%%=*}; envs=${kv#*=}
          env $envs timeout -k 10 300 python3 -u bench.py --model lsgan --no-cpu-baseline > $O/abl_${t}_$i.json 2> $O/abl_${t}_$i.err || exit $?
        done
      done ;;
    gemmtrace)
      t=${arg:-trace}; w=8; [ "$t" != trace ] && w=72
      CGL_PLAN_DEBUG=1 CGL_LIB_PATH=$R/cgl-gan_amd/lib_$t/libcglgan_hip.so timeout -k 10 200 python3 -u tools/gemm_trace.py \
        --words $w --out $O/gemm_trace_$t.json > $O/gemm_trace_$t.log 2>&1 || exit $? ;;
    capprobe)
      timeout -k 10 600 python3 -u tools/capture_probe.py > $O/capture_probe.txt 2>&1 || exit $? ;;
    rccl)
      timeout -k 10 300 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port 29517 tests/rccl_world1_worker.py --time > $O/rccl.log 2>&1 || exit $? ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
echo done > $O/done.txt
