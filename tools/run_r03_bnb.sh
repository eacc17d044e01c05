# cgl_bn_bwd features per workgroup (CGL_BNB_FPW 32 / 16 / 8 / 4): MLP parity tests at the non-default widths,
# bench A/B interleaved (usage: run_r03_bnb.sh "<test widths>" "<bench widths>")
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_bnb
mkdir -p $O
for f in $1; do
  CGL_BNB_FPW=$f timeout -k 10 300 python3 -u -m pytest tests/test_gpu_step.py tests/test_gpu_configs.py tests/test_gpu_ops.py -q --timeout 250 --timeout-method thread > $O/tests_$f.log 2>&1 || exit $?
done
for r in a b; do
  for f in $2; do
    CGL_BNB_FPW=$f timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 400 > $O/bench_f$f$r.json 2> $O/bench_f$f$r.err || exit $?
  done
done
