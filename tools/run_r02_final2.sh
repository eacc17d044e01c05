# round-2 closing evidence: conv round kernel stats + trace, default (MLP) bench line with CPU baseline / parity
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/fin_conv -o run --output-format csv -- python3 -u $R/bench.py --model lsgan --steps 30 --warmup 5 --no-cpu-baseline --profile-reps 1 > $O/fin_conv.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/fin_mlp -o run --output-format csv -- python3 -u $R/bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/fin_mlp_prof.log 2>&1 || exit $?
cd $R
timeout -k 10 300 python3 -u bench.py > $O/fin_mlp.json 2> $O/fin_mlp.err || exit $?
