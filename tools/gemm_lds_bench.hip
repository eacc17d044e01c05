// Microbenchmark: LDS-staged (global_load_lds, full 128-B lines, XOR-swizzled image) fp32 MFMA GEMM
// for k-contiguous operands (NT: C = A B^T, A [M][K], B [N][K]) vs the production cgl_gemm_f32
// (fragment-shaped global loads) on the large shapes of the B=256 round.  Tuning aid.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gemm_lds_bench.hip -o tools/gemm_lds_bench
#include "../cgl-gan_amd/csrc/cgl_gemm.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                         \
      exit(1);                                                                                 \
    }                                                                                          \
  } while (0)

typedef __attribute__((address_space(3))) void lds_void;

// 4 waves as WM x WN x WK: waves of one K-slice (wk) share that slice's LDS ring (A panel 32 WM
// rows, B panel 32 WN rows, BK = 32 per stage, NS stages) filled by global_load_lds_dwordx4; each
// wave owns one 32 x 32 block (two accumulation chains); the WK slices are summed through LDS.
// Stage image per operand panel: rows x 32 k floats, row r's 16-byte piece p stored at piece
// p ^ ((r >> 1) & 7) (conflict-free ds_read_b128).  K split over gridDim.z (partials per z).
template <int WM, int WN, int WK, int NS>
__global__ __launch_bounds__(256) void gemm_lds_nt(const float* __restrict__ A, const float* __restrict__ B,
                                                   float* __restrict__ C, int M, int N, int K, int lda, int ldb,
                                                   int ldc) {
  constexpr int NA = 4 * WM, NB = 4 * WN, NI = NA + NB, GW = WM * WN, PER = NI / GW;
  constexpr int STG = NI * 256;                      // floats per stage per slice
  __shared__ __attribute__((aligned(1024))) float lds[WK * NS * STG];
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int li = lane & 31, lh = lane >> 5;
  const int wk = wave % WK, wmn = wave / WK, wm = wmn / WN, wn = wmn % WN;
  const int m0 = blockIdx.x * 32 * WM, n0 = blockIdx.y * 32 * WN;
  const int nst = K / 32, ks = gridDim.z * WK, sl = blockIdx.z * WK + wk;
  const int sb = (sl * nst) / ks, se = ((sl + 1) * nst) / ks;
  const int cmax = (nst + ks - 1) / ks;
  float* ring = lds + wk * NS * STG;
  const float* src[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int ins = wmn + u * GW;
    const bool isA = ins < NA;
    const int row = (isA ? ins : ins - NA) * 8 + (lane >> 3);
    const int p = (lane & 7) ^ ((row >> 1) & 7);
    const int grow = min((isA ? m0 : n0) + row, (isA ? M : N) - 1);
    src[u] = (isA ? A + (long)grow * lda : B + (long)grow * ldb) + 4 * p;
  }
  auto issue = [&](int s, int buf) {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int ins = wmn + u * GW;
      float* dst = ring + buf * STG + ins * 256;
      __builtin_amdgcn_global_load_lds((const void*)(src[u] + s * 32), (lds_void*)dst, 16, 0, 0);
    }
  };
  typedef float f32x16_ __attribute__((ext_vector_type(16)));
  f32x16_ acc0, acc1;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc0[r] = acc1[r] = 0.f;
  const int arow = wm * 32 + li, brow = wn * 32 + li;
  const int asw = (arow >> 1) & 7, bsw = (brow >> 1) & 7;
  for (int j = 0; j < NS - 1; ++j)
    if (sb + j < se) issue(sb + j, j);
  for (int it = 0; it < cmax; ++it) {
    const int s = sb + it;
    if (s + NS - 2 < se) {
      if constexpr (NS == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
      else if constexpr (NS == 4) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (s + NS - 1 < se) issue(s + NS - 1, (it + NS - 1) % NS);
    if (s < se) {
      const float* la = ring + (it % NS) * STG;
      const float* lb = la + NA * 256;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int p0 = 4 * c + 2 * lh;
        const f32x4 a0 = *(const f32x4*)(la + arow * 32 + 4 * (p0 ^ asw));
        const f32x4 a1 = *(const f32x4*)(la + arow * 32 + 4 * ((p0 + 1) ^ asw));
        const f32x4 b0 = *(const f32x4*)(lb + brow * 32 + 4 * (p0 ^ bsw));
        const f32x4 b1 = *(const f32x4*)(lb + brow * 32 + 4 * ((p0 + 1) ^ bsw));
        const float av[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
        const float bv[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
#pragma unroll
        for (int q = 0; q < 8; q += 2) {
          acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(av[q], bv[q], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(av[q + 1], bv[q + 1], acc1, 0, 0, 0);
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) acc0[r] += acc1[r];
  if constexpr (WK > 1) {     // slices summed through LDS in slice order
    __syncthreads();
    float* red = lds;
    if (wk > 0)
      for (int r = 0; r < 16; ++r) red[((wmn * (WK - 1) + wk - 1) * 16 + r) * 64 + lane] = acc0[r];
    __syncthreads();
    if (wk == 0)
      for (int q = 1; q < WK; ++q)
        for (int r = 0; r < 16; ++r) acc0[r] += red[((wmn * (WK - 1) + q - 1) * 16 + r) * 64 + lane];
  }
  if (wk != 0) return;
  float* Cz = C + (long)blockIdx.z * M * ldc;
  const int col = n0 + wn * 32 + li;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m0 + wm * 32 + 4 * lh + (r & 3) + 8 * (r >> 2);
    if (row < M && col < N) Cz[(long)row * ldc + col] = acc0[r];
  }
}

__global__ void ref_nt(const float* A, const float* B, double* C, int M, int N, int K) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= M * N) return;
  const int m = i / N, n = i % N;
  double s = 0.0;
  for (int k = 0; k < K; ++k) s += (double)A[(long)m * K + k] * B[(long)n * K + k];
  C[i] = s;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 100;
  struct Sh { const char* name; int M, N, K; };
  Sh shapes[] = {{"G4 fwd", 512, 784, 1024}, {"G3 fwd", 512, 1024, 512}, {"D0 fwd", 512, 512, 768},
                 {"E0 fwd", 256, 512, 768}, {"G2 fwd", 512, 512, 256}, {"D1 fwd", 512, 256, 512}};
  const int maxe = 1024 * 1024 * 4;
  float *A, *B, *C, *Cp;
  double* R;
  CglGemmDesc* dd;
  CK(hipMalloc(&A, maxe * 4));
  CK(hipMalloc(&B, maxe * 4));
  CK(hipMalloc(&C, maxe * 4 * 4));
  CK(hipMalloc(&Cp, maxe * 4));
  CK(hipMalloc(&R, maxe * 8));
  CK(hipMalloc(&dd, sizeof(CglGemmDesc)));
  std::vector<float> h(maxe);
  srand(1);
  for (auto& x : h) x = (float)rand() / RAND_MAX * 2.f - 1.f;
  CK(hipMemcpy(A, h.data(), maxe * 4, hipMemcpyHostToDevice));
  for (auto& x : h) x = (float)rand() / RAND_MAX * 2.f - 1.f;
  CK(hipMemcpy(B, h.data(), maxe * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](auto fn) {
    for (int i = 0; i < 10; ++i) fn();
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) fn();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3 / reps;
  };
  for (auto& sh : shapes) {
    const int M = sh.M, N = sh.N, K = sh.K;
    const double gf = 2.0 * M * N * K / 1e9;
    // production kernel (cost-model tile choice)
    CglGemmDesc d;
    memset(&d, 0, sizeof(d));
    d.layout = 0; d.M = M; d.N = N; d.K = K; d.a.split = d.b.split = 0x7fffffff;
    d.a.p0 = A; d.a.ld = K; d.b.p0 = B; d.b.ld = K; d.C = Cp; d.ldc = N; d.a_vec = d.b_vec = 1; d.ksplit = 1;
    // 1x1 tiles, WK = 4 (the plan's choice on these shapes)
    d.TM = d.TN = 1; d.WM = 1; d.WN = 1; d.WK = 4;
    d.tiles_m = (M + 31) / 32; d.tiles_n = (N + 31) / 32;
    CK(hipMemcpy(dd, &d, sizeof(d), hipMemcpyHostToDevice));
    const int g0 = cgl_gemm_wgs(d), sh0 = cgl_gemm_stage_bytes(d);
    const double t0 = timeit([&]() { cgl_gemm_f32<1, 1><<<g0, 256, sh0, 0>>>(dd, 1); });
    printf("%-7s M=%4d N=%4d K=%4d | prod 1x1/WK4 %6.2f us %5.1f TF", sh.name, M, N, K, t0, gf / t0 * 1e3);
    // reference
    ref_nt<<<(M * N + 255) / 256, 256>>>(A, B, R, M, N, K);
    std::vector<double> hr(M * N);
    std::vector<float> hc(M * N * 4);
    CK(hipMemcpy(hr.data(), R, M * N * 8, hipMemcpyDeviceToHost));
    auto run = [&](const char* tag, auto kern, int wm, int wn, int wk, int ks) {
      if ((K / 32) % (ks * wk) && (K / 32) < ks * wk) return;
      dim3 grid((M + 32 * wm - 1) / (32 * wm), (N + 32 * wn - 1) / (32 * wn), ks);
      const double t = timeit([&]() { kern<<<grid, 256, 0, 0>>>(A, B, C, M, N, K, K, K, N); });
      CK(hipMemcpy(hc.data(), C, (size_t)M * N * ks * 4, hipMemcpyDeviceToHost));
      double err = 0, nrm = 0;
      for (int i = 0; i < M * N; ++i) {
        double s = 0;
        for (int z = 0; z < ks; ++z) s += hc[(size_t)z * M * N + i];
        err = fmax(err, fabs(s - hr[i]));
        nrm = fmax(nrm, fabs(hr[i]));
      }
      printf(" | %s ks%d %5.2f us %4.1f TF wg%d e%.0e", tag, ks, t, gf / t * 1e3, grid.x * grid.y * grid.z, err / nrm);
    };
    run("114n2", gemm_lds_nt<1, 1, 4, 2>, 1, 1, 4, 1);
    run("114n3", gemm_lds_nt<1, 1, 4, 3>, 1, 1, 4, 1);
    run("212n3", gemm_lds_nt<2, 1, 2, 3>, 2, 1, 2, 1);
    run("122n3", gemm_lds_nt<1, 2, 2, 3>, 1, 2, 2, 1);
    run("221n3", gemm_lds_nt<2, 2, 1, 3>, 2, 2, 1, 1);
    run("221n3", gemm_lds_nt<2, 2, 1, 3>, 2, 2, 1, 2);
    run("212n3", gemm_lds_nt<2, 1, 2, 3>, 2, 1, 2, 2);
    printf("\n");
  }
  return 0;
}
