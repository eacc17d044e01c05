# A/B of the MLP round: k-loop register-pipeline depth of the 1x1 GEMM waves (variant libraries from
# tools/build_variant.sh) and forced wave arrangements, one box session, default measured first and last.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03_stages
mkdir -p $O
L=$GRAFT_REPO_ROOT/cgl-gan_amd
run() {   # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --steps 400 > $O/$tag.json 2> $O/$tag.err || exit $?
  python3 -c "import json,sys; d=json.load(open('$O/$tag.json')); r=d['roofline']; print('%-10s %.4f ms  gemm %s' % ('$tag', d['ms_per_step'], r['gemm_launch_us']))" >> $O/summary.txt
}
run base0 X=0
for v in s4 s5 s6 s4n1; do run $v CGL_LIB_PATH=$L/lib_$v/libcglgan_hip.so; done
run wk2a CGL_GEMM_TILE=2,1,2,1
run wk2b CGL_GEMM_TILE=1,2,2,1
run base1 X=0
cat $O/summary.txt
