# conv round: weight-gradient operand pipeline depth (CGL_WGRAD_S) A/B, interleaved; variants from
# tools/build_conv_variant.sh selected with CGL_LIB_PATH
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c_wgs
mkdir -p $O
for v in def ws3 ws4 def ws3 ws4; do
  lib=""; [ $v != def ] && lib=$PWD/cgl-gan_amd/lib_$v/libcglgan_hip.so
  CGL_LIB_PATH=$lib timeout -k 10 300 python3 -u bench.py --model lsgan --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || exit $?
  python3 -c "import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', d['ms_per_step'], [(o['op'], o['geom'], o['us']) for o in r['ops'] if o['op']=='wgrad' and o['us']>50])" >> $O/summary.txt
done
