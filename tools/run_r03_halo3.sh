# HALO up-conv extended to the 128-channel conv_blocks.1: halo tests + conv parity suite, lsgan bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_halo3
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_conv_halo.py tests/test_gpu_conv_split_graph.py tests/test_gpu_conv_dist.py tests/test_gpu_conv_multiworker.py tests/test_gpu_conv_step.py tests/test_gpu_conv_bnfold.py tests/test_gpu_conv_ops.py -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for r in a b; do
  for h in 1 0; do
    CGL_CONV_HALO=$h timeout -k 10 200 python3 -u bench.py --model lsgan --no-cpu-baseline --steps 40 > $O/bench_h${h}$r.json 2> $O/bench_h${h}$r.err || exit $?
  done
done
