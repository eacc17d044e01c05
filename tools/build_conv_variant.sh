# Build a variant of libcglgan_hip.so whose conv translation unit gets extra compile definitions:
#   bash tools/build_conv_variant.sh TAG "-DCGL_WGRAD_S=3"   ->  cgl-gan_amd/lib_TAG/libcglgan_hip.so
# (select it with CGL_LIB_PATH; the MLP translation unit is reused from the default build)
set -e
tag=$1; defs=$2
cd "$(dirname "$0")/../cgl-gan_amd"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-result -mllvm -amdgpu-kernarg-preload-count=16"
mkdir -p build lib_$tag
/opt/rocm/bin/hipcc $FLAGS $defs -c csrc/cgl_conv_tu.hip -o build/cvar_$tag.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared build/cgl_runtime.o build/cgl_gemm_p*.o build/cvar_$tag.o \
  -o lib_$tag/libcglgan_hip.so
echo "built lib_$tag ($defs)"
