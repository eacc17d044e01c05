# rocprofv3 kernel stats + PMC traffic passes of the conv round (bench.py --model lsgan)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_conv -o run --output-format csv -- python3 -u $R/bench.py --model lsgan --steps 30 --warmup 5 --no-cpu-baseline > $O/prof_conv.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_conv_fetch -o run --output-format csv -- python3 -u $R/bench.py --model lsgan --steps 10 --warmup 3 --no-cpu-baseline --eager > $O/pmc_conv_fetch.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_conv_write -o run --output-format csv -- python3 -u $R/bench.py --model lsgan --steps 10 --warmup 3 --no-cpu-baseline --eager > $O/pmc_conv_write.log 2>&1 || exit $?
