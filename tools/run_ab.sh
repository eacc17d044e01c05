# GPU tests, then an A/B of the MLP bench under env settings: bash tools/run_ab.sh TAG "ENV=.." TAG2 "ENV=.."
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu ${TESTS:-tests} > $O/ab_gpu.log 2>&1 || exit $?
fi
while [ $# -gt 1 ]; do
  tag=$1; envs=$2; shift 2
  env $envs timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 300 ${BENCH_ARGS} > $O/ab_$tag.json 2> $O/ab_$tag.err || exit $?
done
