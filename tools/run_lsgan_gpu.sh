set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --model lsgan --steps 20 --warmup 3 > gpurun_out/bench_lsgan.json 2> gpurun_out/bench_lsgan.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lsgan -o run -- python -u bench.py --model lsgan --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_lsgan.log 2>&1
