# Build a variant of libcglgan_hip.so with extra compile definitions for an A/B on the box:
#   bash tools/build_variant.sh TAG "-DCGL_GEMM_STAGES1=5"   ->  cgl-gan_amd/lib_TAG/libcglgan_hip.so
# (select it with CGL_LIB_PATH; the conv translation unit is reused from the default build).  The runtime and
# the four GEMM-instantiation translation units are rebuilt with the definitions (in parallel).
set -e
tag=$1; defs=$2
cd "$(dirname "$0")/../cgl-gan_amd"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-result -mllvm -amdgpu-kernarg-preload-count=16"
mkdir -p build lib_$tag
/opt/rocm/bin/hipcc $FLAGS $defs -c csrc/cgl_runtime.hip -o build/var_$tag.o &
for p in 1 2 3 4; do
  /opt/rocm/bin/hipcc $FLAGS $defs -DCGL_GEMM_PART=$p -c csrc/cgl_gemm_inst.hip -o build/var_${tag}_p$p.o &
done
wait
/opt/rocm/bin/hipcc $FLAGS -shared build/var_$tag.o build/var_${tag}_p1.o build/var_${tag}_p2.o build/var_${tag}_p3.o \
  build/var_${tag}_p4.o build/cgl_conv_tu.o -o lib_$tag/libcglgan_hip.so
echo "built lib_$tag ($defs)"
