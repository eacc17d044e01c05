# HALO up-conv: conv parity suite with halo on (default), halo bitwise vs direct, then lsgan bench A/B
# (halo 1/0 x BN fold 2/3, interleaved)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_halo2
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_conv_halo.py tests/test_gpu_conv_step.py tests/test_gpu_conv_bnfold.py tests/test_gpu_conv_ops.py -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for r in a b; do
  for h in 1 0; do
    for f in 2 3; do
      CGL_CONV_HALO=$h CGL_CONV_BNFOLD=$f timeout -k 10 200 python3 -u bench.py --model lsgan --no-cpu-baseline --steps 40 > $O/bench_h${h}f${f}$r.json 2> $O/bench_h${h}f${f}$r.err || exit $?
    done
  done
done
