# Round-end evidence on one MI355X: GPU tests (default plan and split-K plan), the default bench line,
# a rocprofv3 kernel-trace summary of the same command, and the two PMC passes for HBM traffic.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/final_gpu.log 2>&1 || exit $?
CGL_SPLITK=-1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_step.py tests/test_gpu_multiworker.py > $O/final_gpu_splitk.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > $O/bench_final.json 2> $O/bench_final.err || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_final_b.json 2>> $O/bench_final.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mlp -o run --output-format csv -- python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline > $O/prof_mlp.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --eager > $O/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --eager > $O/pmc_write.log 2>&1 || exit $?
