// Microbenchmark of cgl_gemm_f32 on the GEMM shapes of one B=256 CAPGAN round (tuning aid).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gemm_bench.hip -o tools/gemm_bench && tools/gemm_bench
// Prints, per shape and wave arrangement (WM,WN,WK), the mean device time of back-to-back
// launches (hipEvent over 200 launches) and the achieved fp32 TFLOP/s.
#define CGL_GEMM_PART_TU 1   // (device functions of cgl_kernels.hip only: the deferred head finish)
#include "../cgl-gan_amd/csrc/cgl_gemm.hip"
#include "../cgl-gan_amd/csrc/cgl_kernels.hip"

#include <climits>
#include <cmath>
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

__global__ void empty_kernel(int* p) {
  if (p && threadIdx.x == 9999) p[0] = 1;
}

static double time_desc(CglGemmDesc d, CglGemmDesc* dd, int reps) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipMemcpy(dd, &d, sizeof(d), hipMemcpyHostToDevice);
  const int grid = cgl_gemm_wgs(d);
  const int sh = cgl_gemm_stage_bytes(d);
  // one problem: no second / third problem, its layout and vector flags as the selection, no deferred head,
  // no next-launch descriptor warm-up
  const int meta = d.layout | ((d.a_vec && d.b_vec) ? 4 : 0);
  auto go = [&]() {
    if (d.ksplit > 1) {
      if (d.TM == 2)
        cgl_gemm_f32<2, 2, true><<<grid, 256, sh, 0>>>(dd, INT_MAX, INT_MAX, meta, 0, nullptr, 0);
      else
        cgl_gemm_f32<1, 1, true><<<grid, 256, sh, 0>>>(dd, INT_MAX, INT_MAX, meta, 0, nullptr, 0);
    } else if (d.TM == 2) {
      cgl_gemm_f32<2, 2><<<grid, 256, sh, 0>>>(dd, INT_MAX, INT_MAX, meta, 0, nullptr, 0);
    } else {
      cgl_gemm_f32<1, 1><<<grid, 256, sh, 0>>>(dd, INT_MAX, INT_MAX, meta, 0, nullptr, 0);
    }
  };
  for (int i = 0; i < 10; ++i) go();
  (void)hipEventRecord(e0, 0);
  for (int i = 0; i < reps; ++i) go();
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3 / reps;
}

static void probes(float* A, float* B, float* C, float* bias, CglGemmDesc* dd, int reps) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int grid : {1, 256, 1024}) {
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(empty_kernel, dim3(grid), dim3(256), 0, 0, (int*)nullptr);
    (void)hipEventRecord(e0, 0);
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(empty_kernel, dim3(grid), dim3(256), 0, 0, (int*)nullptr);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("probe empty kernel grid=%d: %.2f us/launch\n", grid, ms * 1e3 / reps);
  }
  // hipGraph replay of 28 dependent empty kernels (the per-node floor of a captured round)
  {
    hipStream_t cs;
    CK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    hipGraph_t gr;
    hipGraphExec_t ge;
    for (int grid : {1, 256}) {
      CK(hipStreamBeginCapture(cs, hipStreamCaptureModeGlobal));
      for (int i = 0; i < 28; ++i) hipLaunchKernelGGL(empty_kernel, dim3(grid), dim3(256), 0, cs, (int*)nullptr);
      CK(hipStreamEndCapture(cs, &gr));
      CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
      for (int i = 0; i < 5; ++i) CK(hipGraphLaunch(ge, cs));
      CK(hipStreamSynchronize(cs));
      (void)hipEventRecord(e0, cs);
      for (int i = 0; i < 50; ++i) CK(hipGraphLaunch(ge, cs));
      (void)hipEventRecord(e1, cs);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      printf("probe graph of 28 empty kernels grid=%d: %.2f us/replay (%.2f us/kernel)\n", grid, ms * 1e3 / 50,
             ms * 1e3 / 50 / 28);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(gr));
    }
  }
  // fixed tile count (NT 256x256 -> 64 WGs of (1,1,4)), growing K
  for (int K : {16, 64, 256, 1024, 4096}) {
    for (int wk : {1, 4}) {
      CglGemmDesc d;
      memset(&d, 0, sizeof(d));
      d.layout = 0; d.M = 256; d.N = 256; d.K = K;
      d.WM = 1; d.WN = (wk == 1) ? 4 : 1; d.WK = wk;
      d.tiles_m = 8; d.tiles_n = (wk == 1) ? 2 : 8;
      d.a.p0 = A; d.a.split = 0x7fffffff; d.a.ld = K;
      d.b.p0 = B; d.b.split = 0x7fffffff; d.b.ld = K;
      d.a_vec = d.b_vec = 1;
      d.C = C; d.ldc = 256; d.slope = 0.2f;
      d.TM = d.TN = 1;
      const double us = time_desc(d, dd, reps);
      printf("probe NT 256x256 K=%5d WK=%d WGs=%3d: %7.2f us  (%.1f TF, %d MFMA/wave)\n", K, wk,
             d.tiles_m * d.tiles_n, us, 2.0 * 256 * 256 * K / us * 1e-6, (K / 16 / wk) * 8);
      // same launch with every row of A and B aliased to row 0 (ld = 0): a fragment load then
      // touches 1 cache line instead of 32 -- isolates the per-CU address/L1 cost
      d.a.ld = 0; d.b.ld = 0;
      const double usb = time_desc(d, dd, reps);
      printf("probe NT 256x256 K=%5d WK=%d rows aliased: %7.2f us  (%.1f TF)\n", K, wk, usb,
             2.0 * 256 * 256 * K / usb * 1e-6);
    }
  }
}

// Cost of each fused prologue/epilogue feature on the G-forward shapes (same tiles as the plan).
static void fusion_costs(float* A, float* B, float* C, CglGemmDesc* dd, int reps) {
  float *part, *vec, *cp;
  CK(hipMalloc(&part, 64 * 2 * 1024 * 2 * 4));
  CK(hipMemset(part, 0, 64 * 2 * 1024 * 2 * 4));
  CK(hipMalloc(&vec, 16 * 1024 * 4));
  CK(hipMalloc(&cp, 512 * 1024 * 4));
  std::vector<float> h(16 * 1024, 1.f);
  CK(hipMemcpy(vec, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  const Shape fw[] = {{"G1 fwd", 0, 512, 256, 128}, {"G2 fwd", 0, 512, 512, 256}, {"G3 fwd", 0, 512, 1024, 512},
                      {"G4 fwd", 0, 512, 784, 1024}};
  const int cfg[6][4] = {{2, 1, 2, 1}, {1, 2, 2, 1}, {1, 1, 4, 1}, {2, 1, 2, 2}, {1, 2, 2, 2}, {1, 1, 4, 2}};
  printf("fusion costs (us): plain | +stat partials | +A copy-out\n");
  for (const Shape& s : fw) {
    for (auto& c : cfg) {
      CglGemmDesc d;
      memset(&d, 0, sizeof(d));
      d.layout = 0; d.M = s.M; d.N = s.N; d.K = s.K;
      d.WM = c[0]; d.WN = c[1]; d.WK = c[2]; d.TM = d.TN = c[3];
      d.tiles_m = (s.M + 32 * c[3] * c[0] - 1) / (32 * c[3] * c[0]);
      d.tiles_n = (s.N + 32 * c[3] * c[1] - 1) / (32 * c[3] * c[1]);
      d.a.p0 = A; d.a.split = 0x7fffffff; d.a.ld = s.K;
      d.b.p0 = B; d.b.split = 0x7fffffff; d.b.ld = s.K;
      d.a_vec = d.b_vec = 1;
      d.C = C; d.ldc = s.N; d.slope = 0.2f; d.bias = vec;
      const double t0 = time_desc(d, dd, reps);
      d.stat_part = part; d.stat_gr = 256;
      const double t1 = time_desc(d, dd, reps);
      d.a_copy = cp; d.a_copy_ld = s.K; d.a_copy_row0 = 256;
      const double t2 = time_desc(d, dd, reps);
      printf("%-7s %d%d%d/%d: %7.2f | %7.2f | %7.2f\n", s.name, c[0], c[1], c[2], c[3], t0, t1, t2);
    }
  }
}

// Cross-workgroup split-K: per shape, the (WM,WN,WK)/T arrangements 114/1, 122/1 and 212/1 at
// KS = 1, 2, 4 (results checked against KS = 1).
static void splitk_table(float* A, float* B, float* C, float* bias, CglGemmDesc* dd, int reps) {
  float* kpart;
  unsigned int* kcount;
  CK(hipMalloc(&kpart, (size_t)(4 << 20) * 4));
  CK(hipMalloc(&kcount, 8192 * 4));
  CK(hipMemset(kcount, 0, 8192 * 4));
  const Shape shapes[] = {
      {"G3 fwd", 0, 512, 1024, 512}, {"G4 fwd", 0, 512, 784, 1024}, {"D0 fwd", 0, 512, 512, 784},
      {"D1 fwd", 0, 512, 256, 512},  {"E0 fwd", 0, 256, 512, 784},  {"E1 fwd", 0, 256, 256, 512},
      {"E dXg", 1, 256, 784, 512},   {"G4 dA", 1, 256, 1024, 784},  {"G3 dA", 1, 256, 512, 1024},
      {"G2 dA", 1, 256, 256, 512},   {"D gV1", 2, 256, 513, 512},   {"D gV0", 2, 512, 785, 512},
      {"G gW4", 2, 784, 1025, 256},  {"G gW3", 2, 1024, 513, 256},  {"G gW2", 2, 512, 257, 256},
      {"G gW1", 2, 256, 129, 256},
  };
  const int cfgs[3][4] = {{1, 1, 4, 1}, {1, 2, 2, 1}, {2, 1, 2, 1}};
  printf("split-K   shape      M     N     K |");
  for (auto& c : cfgs) printf(" %d%d%d/%d ks1  ks2  ks4 |", c[0], c[1], c[2], c[3]);
  printf("\n");
  for (const Shape& s : shapes) {
    printf("split-K %-7s %5d %5d %5d |", s.name, s.M, s.N, s.K);
    for (auto& c : cfgs) {
      for (int ks : {1, 2, 4}) {
        CglGemmDesc d;
        memset(&d, 0, sizeof(d));
        d.layout = s.layout; d.M = s.M; d.N = s.N; d.K = s.K;
        d.WM = c[0]; d.WN = c[1]; d.WK = c[2]; d.TM = d.TN = c[3];
        d.tiles_m = (s.M + 32 * c[3] * c[0] - 1) / (32 * c[3] * c[0]);
        d.tiles_n = (s.N + 32 * c[3] * c[1] - 1) / (32 * c[3] * c[1]);
        d.a.p0 = A; d.a.split = 0x7fffffff; d.b.p0 = B; d.b.split = 0x7fffffff;
        if (s.layout == 0) {
          d.a.ld = s.K; d.b.ld = s.K; d.a_vec = d.b_vec = (s.K % 4 == 0); d.bias = bias; d.act = CGL_EPI_ACT_LEAKY;
        } else if (s.layout == 1) {
          d.a.ld = s.K; d.a_vec = (s.K % 4 == 0); d.b.ld = s.N; d.b_vec = (s.N % 4 == 0);
        } else {
          d.a.ld = s.M; d.b.ld = s.N - 1; d.a_vec = (s.M % 4 == 0); d.b_vec = ((s.N - 1) % 4 == 0);
          d.b_ones_col = 1; d.bias_out = bias;
        }
        d.slope = 0.2f; d.C = C; d.ldc = s.layout == 2 ? s.N - 1 : s.N;
        d.ksplit = ks; d.kpart = kpart; d.kcount = kcount;
        const int nch = (s.K + 15) / 16;
        if (ks > 1 && (nch < 2 * c[2] * ks || cgl_gemm_kpart_floats(d) > (4 << 20))) {
          printf("    -");
          continue;
        }
        const size_t n = (size_t)s.M * d.ldc;
        static std::vector<float> r0;
        std::vector<float> r1(n);
        CK(hipMemset(C, 0, n * 4));
        (void)time_desc(d, dd, 1);
        CK(hipDeviceSynchronize());
        if (ks == 1) {
          r0.resize(n);
          CK(hipMemcpy(r0.data(), C, n * 4, hipMemcpyDeviceToHost));
        } else {
          CK(hipMemcpy(r1.data(), C, n * 4, hipMemcpyDeviceToHost));
          double num = 0, den = 0;
          for (size_t i = 0; i < n; ++i) {
            num += (double)(r1[i] - r0[i]) * (r1[i] - r0[i]);
            den += (double)r0[i] * r0[i];
          }
          if (!(num <= 1e-10 * den)) printf(" [MISMATCH %.1e]", sqrt(num / (den + 1e-30)));
        }
        printf(" %5.2f", time_desc(d, dd, reps));
      }
      printf(" |");
    }
    printf("\n");
  }
}

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
      {"L1 conv", 0, 512, 8192, 100},   // (index 23: the conv round's Linear(100, 8192) on [z1; z2])
  };
  const int cfgs[8][4] = {{2, 2, 1, 1}, {2, 1, 2, 1}, {1, 2, 2, 1}, {1, 1, 4, 1},
                          {2, 2, 1, 2}, {2, 1, 2, 2}, {1, 2, 2, 2}, {1, 1, 4, 2}};
  for (const void* fn : {(const void*)cgl_gemm_f32<1, 1>, (const void*)cgl_gemm_f32<2, 2>,
                         (const void*)cgl_gemm_f32<1, 1, true>, (const void*)cgl_gemm_f32<2, 2, true>}) {
    for (int kb : {150, 128, 96, 64}) {
      const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, kb * 1024);
      (void)hipGetLastError();
      if (e == hipSuccess) break;
    }
  }
  const size_t big = 4u << 20;  // floats
  float *A, *B, *C, *bias;
  CK(hipMalloc(&A, big * 4));
  CK(hipMalloc(&B, big * 4));
  CK(hipMalloc(&C, big * 4));
  CK(hipMalloc(&bias, 16384 * 4));
  std::vector<float> h(big);
  for (size_t i = 0; i < big; ++i) h[i] = (float)((i * 2654435761u) % 2001) / 1000.f - 1.f;
  CK(hipMemcpy(A, h.data(), big * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(B, h.data(), big * 4, hipMemcpyHostToDevice));
  CK(hipMemset(bias, 0, 16384 * 4));
  CglGemmDesc* dd;
  CK(hipMalloc(&dd, sizeof(CglGemmDesc)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const bool single = argc > 3;   // gemm_bench REPS single SHAPE CFG: one config only (PMC runs)
  if (argc == 3 && atoi(argv[2]) == 2) {   // gemm_bench REPS 2: the split-K table only
    splitk_table(A, B, C, bias, dd, reps);
    return 0;
  }
  if (!single) {
    probes(A, B, C, bias, dd, reps);
    fusion_costs(A, B, C, dd, reps);
  }
  if (argc == 3) return 0;
  const int only_shape = single ? atoi(argv[3]) : -1;
  const int only_cfg = single && argc > 4 ? atoi(argv[4]) : -1;
  double tot_best = 0, tot_flop = 0;
  printf("%-8s %-3s %5s %5s %5s |", "shape", "L", "M", "N", "K");
  for (auto& c : cfgs) printf(" %d%d%d/%d us TF |", c[0], c[1], c[2], c[3]);
  printf(" best\n");
  int si = -1;
  for (const Shape& s : shapes) {
    ++si;
    if (only_shape >= 0 && si != only_shape) continue;
    printf("%-8s %-3d %5d %5d %5d |", s.name, s.layout, s.M, s.N, s.K);
    double best = 1e30;
    int ci = -1;
    for (auto& c : cfgs) {
      ++ci;
      if (only_cfg >= 0 && ci != only_cfg) continue;
      CglGemmDesc d;
      memset(&d, 0, sizeof(d));
      d.layout = s.layout;
      d.M = s.M;
      d.N = s.N;
      d.K = s.K;
      d.WM = c[0];
      d.WN = c[1];
      d.WK = c[2];
      d.TM = d.TN = c[3];
      d.tiles_m = (s.M + 32 * c[3] * c[0] - 1) / (32 * c[3] * c[0]);
      d.tiles_n = (s.N + 32 * c[3] * c[1] - 1) / (32 * c[3] * c[1]);
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
        d.b_vec = (s.N % 4 == 0);
      } else {
        d.a.ld = s.M;
        d.b.ld = s.N - 1;
        d.a_vec = (s.M % 4 == 0);
        d.b_vec = ((s.N - 1) % 4 == 0);
        d.b_ones_col = 1;
        d.bias_out = bias;
      }
      d.slope = 0.2f;
      d.C = C;
      d.ldc = s.layout == 2 ? s.N - 1 : s.N;
      if (c[3] == 2) {  // verify against the 1x1-block kernel on the same inputs
        const size_t n = (size_t)s.M * d.ldc;
        std::vector<float> r0(n), r1(n);
        CglGemmDesc d0 = d;
        d0.TM = d0.TN = 1;
        d0.tiles_m = (s.M + 32 * c[0] - 1) / (32 * c[0]);
        d0.tiles_n = (s.N + 32 * c[1] - 1) / (32 * c[1]);
        CK(hipMemset(C, 0, n * 4));
        (void)time_desc(d0, dd, 1);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(r0.data(), C, n * 4, hipMemcpyDeviceToHost));
        CK(hipMemset(C, 0, n * 4));
        (void)time_desc(d, dd, 1);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(r1.data(), C, n * 4, hipMemcpyDeviceToHost));
        double num = 0, den = 0;
        for (size_t i = 0; i < n; ++i) {
          num += (double)(r1[i] - r0[i]) * (r1[i] - r0[i]);
          den += (double)r0[i] * r0[i];
        }
        if (!(num <= 1e-10 * den)) printf(" [MISMATCH rel %.2e] ", sqrt(num / (den + 1e-30)));
        if (s.layout == 2 && d.bias_out) { /* bias column compared through C only */ }
      }
      const double us = time_desc(d, dd, reps);
      const double flop = 2.0 * s.M * s.N * s.K;
      printf(" %6.2f %5.1f |", us, flop / us * 1e-6);
      if (us < best) best = us;
    }
    tot_best += best;
    tot_flop += 2.0 * s.M * s.N * s.K;
    printf(" %6.2f\n", best);
  }
  printf("sum of best: %.1f us for %.3f GFLOP -> %.1f TFLOP/s\n", tot_best, tot_flop * 1e-9, tot_flop / tot_best * 1e-6);
  return 0;
}
