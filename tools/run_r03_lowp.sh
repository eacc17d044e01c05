# f16 dynamic loss scaling: the 16-bit GPU tests, the MLP GPU suite (Adam / head / prologue touched), and
# the config-5 bench line with its f16 (loss-scaled) variant
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_lowp
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_lowp.py tests/test_gpu_step.py tests/test_gpu_ops.py tests/test_gpu_configs.py tests/test_model_api.py tests/test_gpu_short_batch.py tests/test_gpu_resume.py -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --model mdgan --no-cpu-baseline --steps 200 > $O/bench_mdgan.json 2> $O/bench_mdgan.err || exit $?
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 300 > $O/bench_mlp.json 2> $O/bench_mlp.err || exit $?
