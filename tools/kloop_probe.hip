// k-loop variants of the MLP GEMM on the round's shapes (design probe for the round-3 GEMM):
//   A  v_mfma_f32_32x32x2f32, 1x1 block per wave, operands row-major (k-contiguous rows): what
//      cgl_gemm_f32 does -- every 16-byte fragment load touches 32 rows
//   B  the same MFMA with both operands in FRAGMENT-PACKED order ([32-row block][16-k chunk][half]
//      [lane][4]): every load instruction reads 1 KB contiguous
//   C  v_mfma_f32_16x16x4f32, 2x2 blocks per wave (same 32x32 wave tile), row-major
//   D  16x16x4, 2x2 blocks, packed ([16-row block][16-k chunk][lane][4])
//   E  32x32x2, 1x1, both operands mn-contiguous (A^T[k][m], B[k][n]): 8 dword loads per operand
//      and chunk, each reading two 128-byte row segments
// Each: 256-thread workgroups, one 32x32 output tile per wave, K split WK ways inside the workgroup
// (LDS reduction), 3 register stages in flight, descriptor by value.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/kloop_probe.hip -o tools/kloop_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(1))) const f32x4* gcf4p;

struct P { const float* A; const float* B; float* C; int M, N, K, WK, tiles_m, tiles_n; };

template <int V>
__global__ __launch_bounds__(256) void kprobe(P p) {
  __shared__ float red[3 * 16 * 64];
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int WK = p.WK, wk = wave % WK, wmn = wave / WK;          // 4 / WK tiles per workgroup
  const int tpw = 4 / WK;
  const int tile = blockIdx.x * tpw + wmn;
  if (tile >= p.tiles_m * p.tiles_n) return;
  const int tm = tile % p.tiles_m, tn = tile / p.tiles_m;
  const int K = p.K, nch = K / 16;
  const int cb = wk * nch / WK, ce = (wk + 1) * nch / WK;
  f32x16 acc = {};
  f32x4 acc4[4] = {};
  const int li = lane & 31, lh = lane >> 5;
  constexpr int S = 3;
  if constexpr (V == 4) {
    // A^T [K][M] (m contiguous), B [K][N] (n contiguous): lane (li, lh) reads k = 16c + 8lh + q
    auto ld = [&](const float* X, int ld_, int m0, int c, float (&v)[8]) {
      const float* r = X + (long)(c * 16 + 8 * lh) * ld_ + m0 + li;
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = ((__attribute__((address_space(1))) const float*)r)[(long)q * ld_];
    };
    float a[S][8], b[S][8];
    for (int s = 0; s < S; ++s) { ld(p.A, p.M, tm * 32, min(cb + s, ce - 1), a[s]); ld(p.B, p.N, tn * 32, min(cb + s, ce - 1), b[s]); }
    int c = cb;
    for (; c + S <= ce; c += S) {
#pragma unroll
      for (int s = 0; s < S; ++s) {
#pragma unroll
        for (int q = 0; q < 8; ++q) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s][q], b[s][q], acc, 0, 0, 0);
        ld(p.A, p.M, tm * 32, min(c + s + S, ce - 1), a[s]);
        ld(p.B, p.N, tn * 32, min(c + s + S, ce - 1), b[s]);
      }
    }
#pragma unroll
    for (int s = 0; s < S - 1; ++s)
      if (c + s < ce)
#pragma unroll
        for (int q = 0; q < 8; ++q) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s][q], b[s][q], acc, 0, 0, 0);
  } else if constexpr (V == 0 || V == 1) {
    // A row-block tm (32 rows), B row-block tn
    auto ld = [&](const float* X, int rb, int c, float (&v)[8]) {
      if (V == 0) {
        const float* r = X + (long)(rb * 32 + li) * K + c * 16 + 8 * lh;
        const f32x4 x = *(gcf4p)r, y = *(gcf4p)(r + 4);
        v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3]; v[4] = y[0]; v[5] = y[1]; v[6] = y[2]; v[7] = y[3];
      } else {
        const float* r = X + ((long)(rb * nch + c) * 2) * 256 + lane * 4;
        const f32x4 x = *(gcf4p)r, y = *(gcf4p)(r + 256);
        v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3]; v[4] = y[0]; v[5] = y[1]; v[6] = y[2]; v[7] = y[3];
      }
    };
    float a[S][8], b[S][8];
    for (int s = 0; s < S; ++s) { ld(p.A, tm, min(cb + s, ce - 1), a[s]); ld(p.B, tn, min(cb + s, ce - 1), b[s]); }
    int c = cb;
    for (; c + S <= ce; c += S) {
#pragma unroll
      for (int s = 0; s < S; ++s) {
#pragma unroll
        for (int q = 0; q < 8; ++q) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s][q], b[s][q], acc, 0, 0, 0);
        ld(p.A, tm, min(c + s + S, ce - 1), a[s]);
        ld(p.B, tn, min(c + s + S, ce - 1), b[s]);
      }
    }
#pragma unroll
    for (int s = 0; s < S - 1; ++s)
      if (c + s < ce)
#pragma unroll
        for (int q = 0; q < 8; ++q) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s][q], b[s][q], acc, 0, 0, 0);
  } else {
    // 16x16x4: lane (row l & 15, quarter l >> 4) holds k = 4 quarter + q of a 16-k chunk
    const int r16 = lane & 15, qd = lane >> 4;
    auto ld = [&](const float* X, int rb16, int c, f32x4& v) {
      if (V == 2) v = *(gcf4p)(X + (long)(rb16 * 16 + r16) * K + c * 16 + 4 * qd);
      else v = *(gcf4p)(X + ((long)(rb16 * nch + c)) * 256 + lane * 4);
    };
    f32x4 a[S][2], b[S][2];
    for (int s = 0; s < S; ++s)
      for (int i = 0; i < 2; ++i) { ld(p.A, tm * 2 + i, min(cb + s, ce - 1), a[s][i]); ld(p.B, tn * 2 + i, min(cb + s, ce - 1), b[s][i]); }
    int c = cb;
    for (; c + S <= ce; c += S) {
#pragma unroll
      for (int s = 0; s < S; ++s) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc4[i * 2 + j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s][i][q], b[s][j][q], acc4[i * 2 + j], 0, 0, 0);
        for (int i = 0; i < 2; ++i) { ld(p.A, tm * 2 + i, min(c + s + S, ce - 1), a[s][i]); ld(p.B, tn * 2 + i, min(c + s + S, ce - 1), b[s][i]); }
      }
    }
#pragma unroll
    for (int s = 0; s < S - 1; ++s)
      if (c + s < ce)
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc4[i * 2 + j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s][i][q], b[s][j][q], acc4[i * 2 + j], 0, 0, 0);
    for (int i = 0; i < 4; ++i) for (int r = 0; r < 4; ++r) acc[i * 4 + r] = acc4[i][r];
  }
  // in-workgroup split-K reduction (fixed order)
  if (WK > 1) {
    if (wk > 0) for (int r = 0; r < 16; ++r) red[((wk - 1) * 16 + r) * 64 + lane] = acc[r];
    __syncthreads();
    if (wk > 0) return;
    for (int q = 1; q < WK; ++q) for (int r = 0; r < 16; ++r) acc[r] += red[((q - 1) * 16 + r) * 64 + lane];
  }
  // store (layout-agnostic checksum store: one float4 per lane x 4, contiguous per tile)
  float* C = p.C + (long)tile * 1024;
  for (int q = 0; q < 4; ++q) *(f32x4*)(C + q * 256 + lane * 4) = f32x4{acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]};
}

int main(int argc, char** argv) {
  struct S { const char* name; int M, N, K; } shapes[] = {
      {"G4 fwd", 512, 784, 1024}, {"G3 fwd", 512, 1024, 512}, {"D0 fwd", 512, 512, 784}, {"G3 dA", 256, 512, 1024},
      {"G4 dA", 256, 1024, 784}, {"D1 fwd", 512, 256, 512}, {"G1 fwd", 512, 256, 128}};
  float *A, *B, *C;
  const long big = 8l << 20;
  CK(hipMalloc(&A, big * 4)); CK(hipMalloc(&B, big * 4)); CK(hipMalloc(&C, big * 4));
  std::vector<float> h(big);
  for (long i = 0; i < big; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  CK(hipMemcpy(A, h.data(), big * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(B, h.data(), big * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int reps = 200;
  const char* vn[] = {"32x32 rowmajor", "32x32 packed", "16x16 2x2 rowmajor", "16x16 2x2 packed", "32x32 mn-contig"};
  for (auto& s : shapes) {
    const int Np = (s.N + 31) / 32 * 32;
    for (int WK : {1, 2, 4}) {
      printf("%-7s M=%4d N=%4d K=%4d WK=%d |", s.name, s.M, s.N, s.K, WK);
      for (int v = 0; v < 5; ++v) {
        P p{A, B, C, s.M, Np, s.K, WK, s.M / 32, Np / 32};
        const int tiles = p.tiles_m * p.tiles_n, tpw = 4 / WK, grid = (tiles + tpw - 1) / tpw;
        auto go = [&]() {
          if (v == 0) kprobe<0><<<grid, 256>>>(p);
          if (v == 1) kprobe<1><<<grid, 256>>>(p);
          if (v == 2) kprobe<2><<<grid, 256>>>(p);
          if (v == 3) kprobe<3><<<grid, 256>>>(p);
          if (v == 4) kprobe<4><<<grid, 256>>>(p);
        };
        for (int i = 0; i < 10; ++i) go();
        CK(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) go();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / reps;
        printf(" %s %6.2f us %5.1f TF |", vn[v], us, 2.0 * s.M * s.N * s.K / us / 1e6);
      }
      printf("\n");
    }
  }
  return 0;
}
