# GEMM epilogue operands issued before the k-loop (CGL_GEMM_EPI_PF, default 1 in lib/; lib_epf0 = 0):
# the whole GPU suite on the default library, then an interleaved A/B of the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c_epf
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gputest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gputest.log; [ $rc -le 1 ] || exit $rc
for v in pf1 pf0 pf1 pf0 pf1 pf0; do
  lib=""; [ $v = pf0 ] && lib=$PWD/cgl-gan_amd/lib_epf0/libcglgan_hip.so
  CGL_LIB_PATH=$lib timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 400 > $O/bench_$v.json 2> $O/bench_$v.err || exit $?
  python3 -c "import json; d=json.load(open('$O/bench_$v.json')); r=d['roofline']; print('$v', d['ms_per_step'], r['per_kind_us_per_round'], r['gemm_launch_us'], d.get('parity',{}).get('pass'))" >> $O/summary.txt
done
