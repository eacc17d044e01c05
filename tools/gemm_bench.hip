// Microbenchmark of cgl_gemm_f32 on the GEMM shapes of one B=256 CAPGAN round (tuning aid).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gemm_bench.hip -o tools/gemm_bench && tools/gemm_bench
// Prints, per shape and wave arrangement (WM,WN,WK), the mean device time of back-to-back
// launches (hipEvent over 200 launches) and the achieved fp32 TFLOP/s.
#include "../cgl-gan_amd/csrc/cgl_gemm.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

struct Shape {
  const char* name;
  int layout, M, N, K;
};

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 200;
  const Shape shapes[] = {
      {"G0 fwd", 0, 512, 128, 100},  {"G1 fwd", 0, 512, 256, 128},  {"G2 fwd", 0, 512, 512, 256},
      {"G3 fwd", 0, 512, 1024, 512}, {"G4 fwd", 0, 512, 784, 1024}, {"D0 fwd", 0, 512, 512, 784},
      {"D1 fwd", 0, 512, 256, 512},  {"E0 fwd", 0, 256, 512, 784},  {"E1 fwd", 0, 256, 256, 512},
      {"D dQ0", 1, 512, 512, 256},   {"E dS0", 1, 256, 512, 256},   {"E dXg", 1, 256, 784, 512},
      {"G4 dA", 1, 256, 1024, 784},  {"G3 dA", 1, 256, 512, 1024},  {"G2 dA", 1, 256, 256, 512},
      {"G1 dA", 1, 256, 128, 256},   {"D gV1", 2, 256, 513, 512},   {"D gV0", 2, 512, 785, 512},
      {"G gW4", 2, 784, 1025, 256},  {"G gW3", 2, 1024, 513, 256},  {"G gW2", 2, 512, 257, 256},
      {"G gW1", 2, 256, 129, 256},   {"G gW0", 2, 128, 101, 256},
  };
  const int cfgs[4][3] = {{2, 2, 1}, {2, 1, 2}, {1, 2, 2}, {1, 1, 4}};
  const size_t big = 4u << 20;  // floats
  float *A, *B, *C, *bias;
  CK(hipMalloc(&A, big * 4));
  CK(hipMalloc(&B, big * 4));
  CK(hipMalloc(&C, big * 4));
  CK(hipMalloc(&bias, 4096 * 4));
  std::vector<float> h(big);
  for (size_t i = 0; i < big; ++i) h[i] = (float)((i * 2654435761u) % 2001) / 1000.f - 1.f;
  CK(hipMemcpy(A, h.data(), big * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(B, h.data(), big * 4, hipMemcpyHostToDevice));
  CK(hipMemset(bias, 0, 4096 * 4));
  CglGemmDesc* dd;
  CK(hipMalloc(&dd, sizeof(CglGemmDesc)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  double tot_best = 0, tot_flop = 0;
  printf("%-8s %-3s %5s %5s %5s |", "shape", "L", "M", "N", "K");
  for (auto& c : cfgs) printf("  %d%d%d us  TF  |", c[0], c[1], c[2]);
  printf(" best\n");
  for (const Shape& s : shapes) {
    printf("%-8s %-3d %5d %5d %5d |", s.name, s.layout, s.M, s.N, s.K);
    double best = 1e30;
    for (auto& c : cfgs) {
      CglGemmDesc d;
      memset(&d, 0, sizeof(d));
      d.layout = s.layout;
      d.M = s.M;
      d.N = s.N;
      d.K = s.K;
      d.WM = c[0];
      d.WN = c[1];
      d.WK = c[2];
      d.tiles_m = (s.M + 32 * c[0] - 1) / (32 * c[0]);
      d.tiles_n = (s.N + 32 * c[1] - 1) / (32 * c[1]);
      d.a.p0 = A;
      d.a.split = 0x7fffffff;
      d.b.p0 = B;
      d.b.split = 0x7fffffff;
      if (s.layout == 0) {
        d.a.ld = s.K;
        d.b.ld = s.K;
        d.a_vec = d.b_vec = (s.K % 4 == 0);
        d.bias = bias;
        d.act = CGL_EPI_ACT_LEAKY;
      } else if (s.layout == 1) {
        d.a.ld = s.K;
        d.a_vec = (s.K % 4 == 0);
        d.b.ld = s.N;
      } else {
        d.a.ld = s.M;
        d.b.ld = s.N - 1;
        d.b_ones_col = 1;
        d.bias_out = bias;
      }
      d.slope = 0.2f;
      d.C = C;
      d.ldc = s.layout == 2 ? s.N - 1 : s.N;
      CK(hipMemcpy(dd, &d, sizeof(d), hipMemcpyHostToDevice));
      const int grid = d.tiles_m * d.tiles_n;
      for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(cgl_gemm_f32, dim3(grid), dim3(256), 0, 0, dd, 1);
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(cgl_gemm_f32, dim3(grid), dim3(256), 0, 0, dd, 1);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / reps;
      const double flop = 2.0 * s.M * s.N * s.K;
      printf("  %6.2f %5.1f |", us, flop / us * 1e-6);
      if (us < best) best = us;
    }
    tot_best += best;
    tot_flop += 2.0 * s.M * s.N * s.K;
    printf(" %6.2f\n", best);
  }
  printf("sum of best: %.1f us for %.3f GFLOP -> %.1f TFLOP/s\n", tot_best, tot_flop * 1e-9, tot_flop / tot_best * 1e-6);
  return 0;
}
