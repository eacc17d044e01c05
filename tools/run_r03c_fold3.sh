# conv round: does folding conv_blocks.2's BatchNorm into the up-convolution pay now that the up-convolution
# stages its input window in LDS (halo path applies the fold once per staged element)?  Interleaved A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c_fold3
mkdir -p $O
for t in fold2 fold3 fold2b fold3b; do
  f=${t:4:1}
  CGL_CONV_BNFOLD=$f timeout -k 10 300 python3 -u bench.py --model lsgan --no-cpu-baseline > $O/bench_$t.json 2> $O/bench_$t.err || exit $?
  python3 -c "import json; d=json.loads(open('$O/bench_$t.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$t', d['ms_per_step'], [(o['geom'], o['us']) for o in r['ops'][:2]])" >> $O/summary.txt
done
