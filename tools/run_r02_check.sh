set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/r1_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > $O/r1_bench_mlp.json 2> $O/r1_bench.err || exit $?
timeout -k 10 300 python -u bench.py --model lsgan --no-cpu-baseline > $O/r1_bench_lsgan.json 2>> $O/r1_bench.err || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_mlp -o run --output-format csv -- python -u $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof_mlp.log 2>&1 || exit $?
