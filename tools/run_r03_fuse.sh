# fused G first-layer weight gradient + G Adam: bitwise test, the MLP GPU suite, RCCL world-1 exchange,
# and the fused prologue + G0 GEMM; then the default bench line and the A/B of both fusions
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_fuse
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_fused_adam.py tests/test_gpu_rccl_world1.py tests/test_gpu_step.py tests/test_gpu_ops.py tests/test_gpu_configs.py tests/test_gpu_short_batch.py tests/test_gpu_resume.py tests/test_gpu_lowp.py tests/test_gpu_multiworker.py tests/test_gpu_mlp_dist.py -v --timeout 270 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/tests.log; [ $rc -le 1 ] || exit $rc
run() { local t=$1; shift; env "$@" timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 400 > $O/bench_$t.json 2> $O/bench_$t.err || exit $?; }
run both X=1
run none CGL_FUSE_GADAM=0 CGL_FUSE_PRO=0
run nopro CGL_FUSE_PRO=0
run noadam CGL_FUSE_GADAM=0
run both2 X=1
