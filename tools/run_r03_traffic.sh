# FETCH_SIZE / WRITE_SIZE passes (one counter per rocprofv3 run) of the MLP bench round (graph replay,
# as bench.py times it) and of the eager conv round, for roofline.traffic at this commit
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_traffic
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $O/mlp_$c -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/mlp_$c.log 2>&1 || exit $?
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $O/conv_$c -o run -- python3 $R/bench.py --model lsgan --steps 4 --warmup 2 --no-cpu-baseline --eager --profile-reps 1 > $O/conv_$c.log 2>&1 || exit $?
done
echo done > $O/done.txt
