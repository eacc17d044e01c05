# round-3 MLP check: k-loop probe, the MLP GPU tests, one default bench line
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_mlp
mkdir -p $O
cd $R
if [ -n "$PROBE" ]; then timeout -k 10 200 tools/kloop_probe > $O/kloop_probe.txt 2>&1 || exit $?; fi
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_step.py tests/test_gpu_ops.py tests/test_model_api.py tests/test_gpu_configs.py tests/test_gpu_multiworker.py tests/test_gpu_lowp.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit $?
