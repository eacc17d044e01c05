# per-dispatch kernel trace of the conv round (one round's timeline) + a short MLP bench line
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tl_conv -o run --output-format csv -- python3 -u $R/bench.py --model lsgan --steps 6 --warmup 2 --no-cpu-baseline --profile-reps 1 > $O/tl_conv.log 2>&1 || exit $?
cd $R
timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/mlp.json 2> $O/mlp.err || exit $?
