# conv G BatchNorm fold: the conv GPU tests, then the conv bench A/B (fold on / off, interleaved)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_bnfold
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_conv_bnfold.py tests/test_gpu_conv_step.py tests/test_gpu_conv_ops.py tests/test_gpu_lsgan_modules.py tests/test_gpu_conv_stats_canary.py tests/test_gpu_conv_dist.py tests/test_gpu_conv_multiworker.py -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -le 1 ] || exit $rc
for t in fold2 fold0 fold3 fold2b fold0b; do
  f=${t:4:1}
  CGL_CONV_BNFOLD=$f timeout -k 10 300 python3 -u bench.py --model lsgan --no-cpu-baseline > $O/bench_$t.json 2> $O/bench_$t.err || exit $?
done
