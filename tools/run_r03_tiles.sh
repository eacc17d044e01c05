# In-situ tile sweep of the MLP round: every freely tiled GEMM forced to one wave arrangement
# WM,WN,WK and block T (CGL_GEMM_TILE), per-launch device times from bench.py's launch profile
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_tiles
mkdir -p $O
cd $R
timeout -k 10 120 python3 bench.py --steps 300 --warmup 30 --no-cpu-baseline > $O/default.json 2> $O/default.err || exit $?
for c in 2,2,1,1 2,1,2,1 1,2,2,1 1,1,4,1 2,2,1,2 2,1,2,2 1,2,2,2 1,1,4,2; do
  CGL_GEMM_TILE=$c timeout -k 10 120 python3 bench.py --steps 300 --warmup 30 --no-cpu-baseline > $O/t$c.json 2> $O/t$c.err || exit $?
done
echo done > $O/done.txt
