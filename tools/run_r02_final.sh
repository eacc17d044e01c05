# Round-2 end-of-round evidence on one MI355X: GPU tests, smoke(), the default bench line (with the CPU
# baseline), the conv line, rocprofv3 kernel stats of both, and the MLP PMC traffic passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/final_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/final_smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > $O/final_bench_mlp.json 2> $O/final_bench.err || exit $?
timeout -k 10 300 python -u bench.py --model lsgan > $O/final_bench_lsgan.json 2>> $O/final_bench.err || exit $?
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/final_prof_mlp -o run --output-format csv -- python3 -u $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/final_prof_mlp.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/final_prof_lsgan -o run --output-format csv -- python3 -u $GRAFT_REPO_ROOT/bench.py --model lsgan --steps 30 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/final_prof_lsgan.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $GRAFT_REPO_ROOT/$O/final_pmc_fetch -o run --output-format csv -- python3 -u $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --eager > $GRAFT_REPO_ROOT/$O/final_pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $GRAFT_REPO_ROOT/$O/final_pmc_write -o run --output-format csv -- python3 -u $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --eager > $GRAFT_REPO_ROOT/$O/final_pmc_write.log 2>&1 || exit $?
