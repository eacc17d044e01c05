// MFMA issue-rate probe (tuning aid): v_mfma_f32_32x32x2_f32 chains with operands in registers.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_probe.hip -o tools/mfma_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NACC>
__global__ __launch_bounds__(256) void chain(float* out, int iters, float seed) {
  f32x16 acc[NACC];
  for (int a = 0; a < NACC; ++a)
    for (int r = 0; r < 16; ++r) acc[a][r] = 0.f;
  float x = seed + threadIdx.x * 1e-7f, y = seed * 0.5f;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int a = 0; a < NACC; ++a) acc[a] = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, acc[a], 0, 0, 0);
  }
  float s = 0.f;
  for (int a = 0; a < NACC; ++a)
    for (int r = 0; r < 16; ++r) s += acc[a][r];
  if (s == 12345.f) out[threadIdx.x] = s;
}

template <int NACC>
void run(float* out, int wgs) {
  const int iters = 2048 / NACC;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  chain<NACC><<<wgs, 256>>>(out, iters, 1.f);
  (void)hipEventRecord(e0, 0);
  for (int k = 0; k < 10; ++k) chain<NACC><<<wgs, 256>>>(out, iters, 1.f);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double us = ms * 1e3 / 10;
  const double mfma_per_wave = 8.0 * iters * NACC;
  // cycles per MFMA per wave at 2.4 GHz (waves per SIMD = wgs/256 when wgs >= 256)
  printf("acc=%d wgs=%4d: %8.2f us, %.1f ns per MFMA per wave, %.1f TF\n", NACC, wgs, us, us * 1e3 / mfma_per_wave,
         wgs * 4.0 * mfma_per_wave * 4096.0 / us * 1e-6);
}

int main() {
  float* out;
  (void)hipMalloc(&out, 4096);
  for (int wgs : {256, 512, 1024}) {
    run<1>(out, wgs);
    run<2>(out, wgs);
    run<4>(out, wgs);
  }
  return 0;
}
