// fp32 MFMA GEMM for the MLP GAN step (gfx950, v_mfma_f32_32x32x2_f32).
//
// Replaces the reference's implicit cuBLAS addmm / mm calls of nn.Linear forward and
// autograd backward (model/mnist_model.py:11,22,77,79,81).
//
// Design (MI355X-first, not a CUDA tiling):
//  * one wave owns a 32x32 output tile = ONE f32 MFMA accumulator (16 AGPR/VGPR per lane);
//    v_mfma_f32_32x32x2_f32 issues every 64 cycles with a 64-cycle dependent latency, so a
//    single accumulation chain already runs at the f32 matrix peak;
//  * a 256-thread workgroup holds 4 waves arranged WM x WN x WK: WK > 1 splits K inside the
//    workgroup (skinny, batch-256 GEMMs need it to put >= 1024 waves on the 256 CUs) and the
//    split is summed through LDS in a fixed order (deterministic, no atomics);
//  * operands are loaded straight into the MFMA fragment registers.  The k index of the
//    32x32x2 fragment is permuted so that lane half h owns 8 CONSECUTIVE k of every 16-k
//    chunk: a k-contiguous operand is then two float4 loads per lane per 8 MFMAs;
//  * prologue fusion: the A operand can be the pre-BatchNorm output of the previous layer;
//    the workgroup combines the producer's {sum, M2} partials into a scale/shift table in LDS and applies
//    BatchNorm1d(train) + LeakyReLU while loading (the reference's BN/LeakyReLU kernels
//    disappear), optionally writing the transformed rows out once;
//  * epilogue fusion: bias, LeakyReLU / Tanh, LeakyReLU' mask, Tanh' (1 - t^2), the
//    bias-gradient column (B's extra all-ones column), and per-column {sum, M2} partials of
//    the stored output for the next layer's BatchNorm, grouped per forward call.
#include "cgl_internal.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ const float* cgl_row(const CglRowSrc& s, int r) {
  if (r < s.split) {
    int rr = r;
    if (s.idx0) rr = gldi(s.idx0 + (s.idx_off ? gldi(s.idx_off) : 0) + r);
    return s.p0 + (long)rr * s.ld;
  }
  return s.p1 + (long)(r - s.split) * s.ld;
}

// Loads are issued UNCONDITIONALLY from clamped (always valid) addresses and masked only when
// the values are consumed: a predicated "load or zero" compiles to a branch around every load
// with a full vmcnt(0) drain, which serialises the memory pipeline (measured: one full memory
// latency per 16-k chunk).

// Operand pointers come out of the descriptor in memory, so the compiler cannot prove they are
// global and would emit flat_load_* -- which return out of order and force
// s_waitcnt vmcnt(0) lgkmcnt(0) at every use.  Casting to address space 1 gives global_load_*
// with counted waits.
// raw: 8 consecutive k of one row of a k-contiguous operand (k clamped into [0, K))
template <int VEC>
__device__ __forceinline__ void cgl_ld_kc(const float* __restrict__ rp_, int k, int K, float v[8]) {
  gcfp rp = (gcfp)rp_;
  if (VEC) {  // K % 4 == 0, 16-byte aligned rows
    const f32x4 x = *(gcf4p)(rp + min(k, K - 4));
    const f32x4 y = *(gcf4p)(rp + min(k + 4, K - 4));
    v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
    v[4] = y[0]; v[5] = y[1]; v[6] = y[2]; v[7] = y[3];
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = rp[min(k + j, K - 1)];
  }
}

// raw: rows k..k+7 (clamped) at one column of a row-major [K][ld] (mn-contiguous) operand
__device__ __forceinline__ void cgl_ld_mn(const float* __restrict__ p_, int ld, int k, int K, float v[8]) {
  gcfp p = (gcfp)p_;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = p[(long)min(k + j, K - 1) * ld];
}

__device__ __forceinline__ void cgl_mask(float v[8], bool ok, int k, int K) {
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (ok && k + j < K) ? v[j] : 0.f;
}

// BatchNorm statistics of group g for Q features k[q] (k[q] < 0: unused) from the producer
// partials: the exact parallel combination of per-tile {S_t, M2_t} over c_t rows, in double
// like torch's CPU kernel and in a fixed tile order,
//   mean = sum_t S_t / n,   M2 = sum_t (M2_t + c_t (S_t / c_t - mean)^2).
// Fast path (<= 8 tiles per group): every {S_t, M2_t} pair of the Q features is loaded up front
// as one 8-byte load, so the whole computation costs a single memory round trip.
template <int Q>
__device__ __forceinline__ void cgl_bn_stats(const CglBnFwd& bn, int K, const int (&k)[Q], int g, double (&mean)[Q],
                                             double (&m2)[Q], int& n) {
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  const int r0 = g * bn.gr, r1 = min(r0 + bn.gr, bn.mtot);
  n = r1 - r0;
  const int t0 = r0 / bn.part_bm, t1 = (r1 - 1) / bn.part_bm;
  const int nt = t1 - t0 + 1;
  if (nt <= 8) {
    f32x2 pr[Q][8];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int kk = max(k[q], 0);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int t = t0 + min(j, nt - 1);
        const int slot = (t * bn.part_bm < r0) ? 1 : 0;   // tile starts in the previous group
        pr[q][j] = *(const CGL_GLOBAL f32x2*)(bn.part + ((long)(t * 2 + slot) * K + kk) * 2);
      }
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      double s = 0.0;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (j < nt) s += (double)pr[q][j][0];
      const double mu = s / n;
      double acc = 0.0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (j < nt) {
          const int t = t0 + j;
          const int c = min((t + 1) * bn.part_bm, r1) - max(t * bn.part_bm, r0);
          const double dd = (double)pr[q][j][0] / c - mu;
          acc += (double)pr[q][j][1] + c * dd * dd;
        }
      }
      mean[q] = mu;
      m2[q] = acc;
    }
    return;
  }
  for (int q = 0; q < Q; ++q) {
    const int kk = max(k[q], 0);
    double s = 0.0;
    for (int t = t0; t <= t1; ++t) {
      const int slot = (t * bn.part_bm < r0) ? 1 : 0;
      s += (double)gld(bn.part + ((long)(t * 2 + slot) * K + kk) * 2);
    }
    const double mu = s / n;
    double acc = 0.0;
    for (int t = t0; t <= t1; ++t) {
      const int slot = (t * bn.part_bm < r0) ? 1 : 0;
      const float* pp = bn.part + ((long)(t * 2 + slot) * K + kk) * 2;
      const int c = min((t + 1) * bn.part_bm, r1) - max(t * bn.part_bm, r0);
      const double dd = (double)gld(pp) / c - mu;
      acc += (double)gld(pp + 1) + c * dd * dd;
    }
    mean[q] = mu;
    m2[q] = acc;
  }
}

// Saved statistics (for the backward pass) and running statistics of the 64-feature block
// `blk`, every group in the order of the reference's forward calls (Xd then Xg,
// capgan.py:215-220): torch's momentum update with the unbiased variance.
__device__ void cgl_bn_block_side(const CglBnFwd& bn, int K, int blk) {
  __shared__ double s_mean[2][64], s_m2[2][64];
  __shared__ int s_n[2];
  const int ngroups = (bn.mtot + bn.gr - 1) / bn.gr;   // <= 2
  const int tid = threadIdx.x;
  if (tid < 64 * ngroups) {
    const int g = tid >> 6, c = tid & 63;
    const int kk = blk * 64 + c;
    const int k[1] = {kk < K ? kk : -1};
    double mean[1], m2[1];
    int n;
    cgl_bn_stats<1>(bn, K, k, g, mean, m2, n);
    s_mean[g][c] = mean[0];
    s_m2[g][c] = m2[0];
    if (c == 0) s_n[g] = n;
    if (kk < K && bn.save_mean) {
      gst(bn.save_mean + (long)g * K + kk, (float)mean[0]);
      gst(bn.save_invstd + (long)g * K + kk, (float)(1.0 / sqrt(m2[0] / n + bn.eps)));
    }
  }
  __syncthreads();
  const int kk = blk * 64 + tid;
  if (bn.run_mean && tid < 64 && kk < K) {
    const double mom = bn.momentum;
    float rm = gld(bn.run_mean + kk), rv = gld(bn.run_var + kk);
    for (int g = 0; g < ngroups; ++g) {
      rm = (float)(mom * s_mean[g][tid] + (1.0 - mom) * (double)rm);
      rv = (float)(mom * (s_m2[g][tid] / (s_n[g] - 1)) + (1.0 - mom) * (double)rv);
    }
    gst(bn.run_mean + kk, rm);
    gst(bn.run_var + kk, rv);
  }
}

// ------------------------------------------------------------------------------------------
// LDS-staged main loop (PIPE == 1).
//
// Each k-group of WM x WN waves stages 32-deep k slices of its A panel (32*WM rows) and B panel
// (32*WN columns) through LDS, double buffered: the coalesced global loads of slice s+1
// (every wave-instruction reads whole 128-byte rows: 8 rows x 128 B for a k-contiguous operand)
// are in flight while slice s is consumed from LDS, and each element is loaded once per
// workgroup instead of once per wave that needs it.
//   k-contiguous panel ([row][k], A of NT/NN and B of NT): rows padded to 36 floats, so the
//     fragment reads (ds_read_b128 of 4 consecutive k for 32 rows) are bank-conflict free;
//   mn-contiguous panel ([k][col], A of TN, B of NN/TN): rows of 32*W floats, fragment reads are
//     ds_read_b32 of 32 consecutive columns (conflict free).
// Tails (rows >= M, cols >= N, k >= K) are zero-filled at staging, so the MFMAs need no masks.
// The BatchNorm+LeakyReLU transform of A and its copy-out are applied once, at staging.
constexpr int CGL_BK = 32;
constexpr int CGL_LDK = 36;

__device__ __forceinline__ int cgl_lds_stage_floats(int WM, int WN) { return (32 * WM + 32 * WN) * CGL_LDK; }

template <int LAYOUT, int VEC>
__device__ __forceinline__ void cgl_mainloop_lds(const CglGemmDesc* __restrict__ d, f32x16& acc,
                                                 const float* __restrict__ s_tf, float* __restrict__ s_stage,
                                                 int M, int N, int K, int nmem, int b_ones, int WM, int WN, int WK,
                                                 int wk, int wmn, int wm, int wn, int tm, int tn, int lane, int g0,
                                                 int a_tf) {
  const int gw = WM * WN;
  const int BMr = 32 * WM, BNr = 32 * WN;
  const int a_fl = BMr * CGL_LDK;
  const int stage_fl = cgl_lds_stage_floats(WM, WN);
  float* __restrict__ grp = s_stage + wk * 2 * stage_fl;
  const int nst = (K + CGL_BK - 1) / CGL_BK;
  const int nsg = (nst + WK - 1) / WK;
  const int sb = (wk * nst) / WK, cnt = ((wk + 1) * nst) / WK - sb;
  const int ninst = (4 * WM + 4 * WN) / gw;  // staging wave-instructions per wave per slice (4..8)
  const int arow0 = tm * BMr;                 // first A row (kc) / column (mn) of the panel
  const int bcol0 = tn * BNr;                 // first B row (NT) / column (NN, TN) of the panel
  const int li = lane & 31, lh = lane >> 5;
  const float slope_tf = d->bn.slope;
  const int gr = a_tf ? d->bn.gr : 1;
  float* __restrict__ a_copy = (LAYOUT != 2 && tn == 0) ? d->a_copy : nullptr;
  const int a_copy_ld = d->a_copy_ld, a_copy_row0 = d->a_copy_row0;
  const int lda = d->a.ld, ldb = d->b.ld;

  f32x4 rg[8];  // staging registers (ninst <= 8)

  // address of staging instruction q of this wave for slice s; fills rg[q]
  auto stage_load = [&](int s, int q) {
    const int t = wmn + q * gw;
    const bool isA = t < 4 * WM;
    const int u = isA ? t : t - 4 * WM;
    const bool kc = isA ? (LAYOUT != 2) : (LAYOUT == 0);
    f32x4 v;
    if (kc) {
      const int lrow = 8 * u + (lane >> 3);
      const int k = s * CGL_BK + 4 * (lane & 7);
      const int nrows = isA ? M : N;
      const int grow = min((isA ? arow0 : bcol0) + lrow, nrows - 1);
      const float* rp = cgl_row(isA ? d->a : d->b, grow);
      if (VEC) {
        v = *(gcf4p)(rp + min(k, K - 4));
      } else {
        gcfp g = (gcfp)rp;
        v = f32x4{g[min(k, K - 1)], g[min(k + 1, K - 1)], g[min(k + 2, K - 1)], g[min(k + 3, K - 1)]};
      }
    } else {
      const int R = isA ? BMr : BNr;
      const int lpr = R >> 2;                 // lanes per k-row
      const int rpi = 64 / lpr;               // k-rows per instruction
      const int kl = u * rpi + lane / lpr;
      const int col = (isA ? arow0 : bcol0) + 4 * (lane % lpr);
      const int ncols = isA ? M : nmem;
      const int k = min(s * CGL_BK + kl, K - 1);
      const float* base = (isA ? d->a.p0 : d->b.p0) + (long)k * (isA ? lda : ldb);
      if (VEC && ncols >= 4) {
        v = *(gcf4p)(base + min(col, ncols - 4));
      } else {
        gcfp g = (gcfp)base;
        const int cm = max(ncols - 1, 0);
        v = f32x4{g[min(col, cm)], g[min(col + 1, cm)], g[min(col + 2, cm)], g[min(col + 3, cm)]};
      }
    }
    rg[q] = v;
  };

  // mask / transform / copy-out, then write rg[q] into LDS buffer `buf`
  auto stage_store = [&](int s, int q, float* buf) {
    const int t = wmn + q * gw;
    const bool isA = t < 4 * WM;
    const int u = isA ? t : t - 4 * WM;
    const bool kc = isA ? (LAYOUT != 2) : (LAYOUT == 0);
    f32x4 v = rg[q];
    if (kc) {
      const int lrow = 8 * u + (lane >> 3);
      const int k = s * CGL_BK + 4 * (lane & 7);
      const int nrows = isA ? M : N;
      const int growu = (isA ? arow0 : bcol0) + lrow;
      const bool rok = growu < nrows;
      if (isA && a_tf) {
        const int gsel = rok ? growu / gr - g0 : 0;
        const float* tb = s_tf + (gsel * CGL_TF_MAXK) * 2;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int kk = min(k + j, K - 1);
          const float x = fmaf(v[j], tb[kk * 2 + 0], tb[kk * 2 + 1]);
          v[j] = x > 0.f ? x : x * slope_tf;
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = (rok && k + j < K) ? v[j] : 0.f;
      if (isA && a_copy && rok && growu >= a_copy_row0) {
        float* dst = a_copy + (long)growu * a_copy_ld + k;
        if (VEC && k + 3 < K) {
          *(gf4p)dst = v;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (k + j < K) gst(dst + j, v[j]);
        }
      }
      *reinterpret_cast<f32x4*>(buf + (isA ? 0 : a_fl) + lrow * CGL_LDK + 4 * (lane & 7)) = v;
    } else {
      const int R = isA ? BMr : BNr;
      const int lpr = R >> 2;
      const int rpi = 64 / lpr;
      const int kl = u * rpi + lane / lpr;
      const int cl = 4 * (lane % lpr);
      const int col = (isA ? arow0 : bcol0) + cl;
      const int ncols = isA ? M : nmem;
      const bool kok = s * CGL_BK + kl < K;
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = (kok && col + j < ncols) ? v[j] : 0.f;
      *reinterpret_cast<f32x4*>(buf + (isA ? 0 : a_fl) + kl * R + cl) = v;
    }
  };

  // fragments of sub-chunk j2 (16 k) from LDS buffer `buf`, then 8 MFMAs
  auto compute = [&](int s, const float* buf) {
#pragma unroll
    for (int j2 = 0; j2 < 2; ++j2) {
      float av[8], bv[8];
      const int kq = 16 * j2 + 8 * lh;
      if (LAYOUT != 2) {
        const float* p = buf + (wm * 32 + li) * CGL_LDK + kq;
        const f32x4 x = *reinterpret_cast<const f32x4*>(p);
        const f32x4 y = *reinterpret_cast<const f32x4*>(p + 4);
        av[0] = x[0]; av[1] = x[1]; av[2] = x[2]; av[3] = x[3];
        av[4] = y[0]; av[5] = y[1]; av[6] = y[2]; av[7] = y[3];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) av[j] = buf[(kq + j) * BMr + wm * 32 + li];
      }
      const float* bb = buf + a_fl;
      if (LAYOUT == 0) {
        const float* p = bb + (wn * 32 + li) * CGL_LDK + kq;
        const f32x4 x = *reinterpret_cast<const f32x4*>(p);
        const f32x4 y = *reinterpret_cast<const f32x4*>(p + 4);
        bv[0] = x[0]; bv[1] = x[1]; bv[2] = x[2]; bv[3] = x[3];
        bv[4] = y[0]; bv[5] = y[1]; bv[6] = y[2]; bv[7] = y[3];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) bv[j] = bb[(kq + j) * BNr + wn * 32 + li];
        if (b_ones && bcol0 + wn * 32 + li == N - 1) {
#pragma unroll
          for (int j = 0; j < 8; ++j) bv[j] = (s * CGL_BK + kq + j < K) ? 1.f : 0.f;
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j], bv[j], acc, 0, 0, 0);
    }
  };

  // (staging loops are fully unrolled to 8 with a uniform predicate so rg[] stays in VGPRs)
  // prologue: slice sb into buffer 0
  if (cnt > 0) {
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (q < ninst) stage_load(sb, q);
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (q < ninst) stage_store(sb, q, grp);
  }
  __syncthreads();
  for (int i = 0; i < nsg; ++i) {
    float* cur = grp + (i & 1) * stage_fl;
    float* nxt = grp + ((i + 1) & 1) * stage_fl;
    const bool more = i + 1 < cnt;
    if (more) {
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (q < ninst) stage_load(sb + i + 1, q);
    }
    if (i < cnt) compute(sb + i, cur);
    if (more) {
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (q < ninst) stage_store(sb + i + 1, q, nxt);
    }
    __syncthreads();
  }
}

template <int LAYOUT, int VEC, int PIPE>
__device__ __forceinline__ void cgl_gemm_body(const CglGemmDesc* __restrict__ d, int bid, float* __restrict__ s_tf,
                                              float* __restrict__ s_stage, float* __restrict__ s_col) {
  float* __restrict__ s_red = s_stage;   // split-K partials reuse the staging region after the loop
  const int M = d->M, N = d->N, K = d->K;
  const int WN = d->WN, WK = d->WK, WM = d->WM;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int li = lane & 31, lh = lane >> 5;
  const int wk = wave % WK, wmn = wave / WK;
  const int wm = wmn / WN, wn = wmn % WN;
  // XCD-aware tile order (blocks b and b+8 land on the same XCD): each XCD takes a contiguous
  // range of tiles in n-major order, so its L2 holds ~1/8 of the B panels (the weights) plus
  // the A panels, instead of all of both.  Bijective for any tile count (guide T1).
  const int local = bid - d->wg_begin;
  const int nwg = d->tiles_m * d->tiles_n;
  int tile = local;
  if (nwg >= 16) {
    const int xcd = local & 7, pos = local >> 3, q = nwg >> 3, r = nwg & 7;
    tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
  }
  const int tn = tile / d->tiles_m, tm = tile % d->tiles_m;
  const int BM = 32 * WM;
  const int m0 = tm * BM + wm * 32;
  const int n0 = (tn * WN + wn) * 32;

  // ---------------- BatchNorm prologue: scale/shift pairs of the group(s) of this row tile,
  // four features per thread with one memory round trip; pairs past K (up to the next
  // multiple of 8) are zero, so the transform of a clamped tail load is 0
  const int a_tf = (LAYOUT != 2) ? d->a_tf : 0;
  int g0 = 0;
  if (a_tf) {
    const CglBnFwd& bn = d->bn;
    const int rlast = min(tm * BM + BM, M) - 1;
    g0 = (tm * BM) / bn.gr;
    const int g1 = rlast / bn.gr;
    const int Kp = (K + 7) & ~7;
    for (int g = g0; g <= g1; ++g) {
      float* dst = s_tf + (g - g0) * CGL_TF_MAXK * 2;
      for (int kb = 0; kb < Kp; kb += 4 * CGL_GEMM_THREADS) {
        int k[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) k[q] = (kb + q * CGL_GEMM_THREADS + tid < K) ? kb + q * CGL_GEMM_THREADS + tid : -1;
        double mean[4], m2[4];
        int n;
        cgl_bn_stats<4>(bn, K, k, g, mean, m2, n);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int kk = kb + q * CGL_GEMM_THREADS + tid;
          if (kk < Kp) {
            float sc = 0.f, sh = 0.f;
            if (k[q] >= 0) {
              const double invstd = 1.0 / sqrt(m2[q] / n + bn.eps);
              sc = (float)invstd * gld(bn.gamma + kk);
              sh = gld(bn.beta + kk) - (float)mean[q] * sc;
            }
            dst[2 * kk] = sc;
            dst[2 * kk + 1] = sh;
          }
        }
      }
    }
    // saved / running statistics: 64-feature blocks spread over the first workgroups
    if (bn.run_mean || bn.save_mean) {
      const int nblk = (K + 63) / 64;
      for (int blk = local; blk < nblk; blk += nwg) cgl_bn_block_side(bn, K, blk);
    }
    __syncthreads();
  }

  // ---------------- main loop
  const int b_ones = (LAYOUT != 0) ? d->b_ones_col : 0;
  const int nmem = N - b_ones;     // columns of B actually in memory
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;

  if constexpr (PIPE == 1) {
    cgl_mainloop_lds<LAYOUT, VEC>(d, acc, s_tf, s_stage, M, N, K, nmem, b_ones, WM, WN, WK, wk, wmn, wm, wn, tm, tn,
                                  lane, g0, a_tf);
  } else {
  const int nch = (K + CGL_GEMM_KCHUNK - 1) / CGL_GEMM_KCHUNK;
  const int cb = (wk * nch) / WK, ce = ((wk + 1) * nch) / WK;

  // per-lane operand rows / columns
  const int am = m0 + li;          // A row (kc) or A column (mn)
  const int bn_ = n0 + li;         // B row (NT) or B column (NN/TN)
  const bool a_ok = am < M;
  const bool b_ok = bn_ < nmem;
  const bool b_is_ones = b_ones && (bn_ == N - 1);
  // clamped (always dereferenceable) operand bases
  const float* __restrict__ a_base = (LAYOUT != 2) ? cgl_row(d->a, min(am, M - 1)) : d->a.p0 + min(am, M - 1);
  const float* __restrict__ b_base =
      (LAYOUT == 0) ? cgl_row(d->b, min(bn_, N - 1)) : d->b.p0 + max(0, min(bn_, nmem - 1));
  const int lda = d->a.ld, ldb = d->b.ld;
  const int gsel = a_tf ? (a_ok ? am / d->bn.gr - g0 : 0) : 0;
  const float slope_tf = d->bn.slope;
  float* __restrict__ a_copy = d->a_copy;
  const bool do_copy = (LAYOUT != 2) && a_copy && tn == 0 && wn == 0 && a_ok && am >= d->a_copy_row0;

  auto load_chunk = [&](int c, float* A_, float* B_) {
    const int k = c * CGL_GEMM_KCHUNK + 8 * lh;
    if (LAYOUT == 2)
      cgl_ld_mn(a_base, lda, k, K, A_);
    else
      cgl_ld_kc<VEC>(a_base, k, K, A_);
    if (LAYOUT == 0)
      cgl_ld_kc<VEC>(b_base, k, K, B_);
    else
      cgl_ld_mn(b_base, ldb, k, K, B_);
  };
  auto compute_chunk = [&](int c, float* A_, float* B_) {
    const int k = c * CGL_GEMM_KCHUNK + 8 * lh;
    cgl_mask(A_, a_ok, k, K);
    if (b_is_ones) {
#pragma unroll
      for (int j = 0; j < 8; ++j) B_[j] = (k + j < K) ? 1.f : 0.f;
    } else {
      cgl_mask(B_, b_ok, k, K);
    }
    if (a_tf) {
      // {scale, shift} of k..k+7 (k % 8 == 0): four 16-byte LDS reads, zero pairs past K
      const f32x4* t4 = (const f32x4*)(s_tf + (gsel * CGL_TF_MAXK + k) * 2);
      const f32x4 p0 = t4[0], p1 = t4[1], p2 = t4[2], p3 = t4[3];
      const float sc[8] = {p0[0], p0[2], p1[0], p1[2], p2[0], p2[2], p3[0], p3[2]};
      const float sh[8] = {p0[1], p0[3], p1[1], p1[3], p2[1], p2[3], p3[1], p3[3]};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float x = fmaf(A_[j], sc[j], sh[j]);
        A_[j] = a_ok ? (x > 0.f ? x : x * slope_tf) : 0.f;
      }
    }
    if (do_copy) {
      float* dst = a_copy + (long)am * d->a_copy_ld;
      if (VEC && k + 7 < K) {
        *(gf4p)(dst + k) = f32x4{A_[0], A_[1], A_[2], A_[3]};
        *(gf4p)(dst + k + 4) = f32x4{A_[4], A_[5], A_[6], A_[7]};
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (k + j < K) gst(dst + k + j, A_[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A_[j], B_[j], acc, 0, 0, 0);
  };

  // three register sets in rotation: the loads of chunks c+1 and c+2 are in flight while chunk
  // c's MFMAs run (~2 x 512 MFMA cycles of cover for an L2/MALL miss), and no register copy
  // forces an early wait.  Tail loads are clamped re-loads.
  if (cb < ce) {
    float xa[8], xb[8], ya[8], yb[8], za[8], zb[8];
    load_chunk(cb, xa, xb);
    load_chunk(min(cb + 1, ce - 1), ya, yb);
    for (int c = cb; c < ce; c += 3) {
      load_chunk(min(c + 2, ce - 1), za, zb);
      compute_chunk(c, xa, xb);
      load_chunk(min(c + 3, ce - 1), xa, xb);
      if (c + 1 < ce) compute_chunk(c + 1, ya, yb);
      load_chunk(min(c + 4, ce - 1), ya, yb);
      if (c + 2 < ce) compute_chunk(c + 2, za, zb);
    }
  }
  }  // PIPE == 0

  // ---------------- split-K reduction (fixed order: wk = 1, 2, 3)
  if (WK > 1) {
    if (wk > 0) {
      float* dst = s_red + ((wmn * (WK - 1) + (wk - 1)) * 16) * 64;
#pragma unroll
      for (int r = 0; r < 16; ++r) dst[r * 64 + lane] = acc[r];
    }
    __syncthreads();
    if (wk == 0) {
      for (int q = 1; q < WK; ++q) {
        const float* src = s_red + ((wmn * (WK - 1) + (q - 1)) * 16) * 64;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] += src[r * 64 + lane];
      }
    }
  }

  // ---------------- epilogue (waves with wk == 0 own the tile)
  const bool owner = (wk == 0);
  const int col = n0 + li;
  const bool colok = col < N;
  const bool ones_col = b_ones && col == N - 1;
  float v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = acc[r];
  const int rbase = m0 + 4 * lh;   // row of register r: rbase + (r & 3) + 8 * (r >> 2)

  if (owner && colok && !ones_col) {
    if (d->bias) {
      const float bb = gld(d->bias + col);
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] += bb;
    }
    if (d->act == CGL_EPI_ACT_LEAKY) {
      const float sl = d->slope;
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * sl;
    } else if (d->act == CGL_EPI_ACT_TANH) {
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = tanhf(v[r]);
    }
    if (d->mask_ref) {
      const float sl = d->slope;
      float ref[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = min(rbase + (r & 3) + 8 * (r >> 2), M - 1);
        ref[r] = gld(d->mask_ref + (long)row * d->mask_ld + col);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = ref[r] > 0.f ? v[r] : v[r] * sl;
    }
    if (d->tanh_ref) {
      float t[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = min(rbase + (r & 3) + 8 * (r >> 2), M - 1);
        t[r] = gld(d->tanh_ref + (long)row * d->tanh_ld + col);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = v[r] * (1.f - t[r] * t[r]);
    }
  }

  // forward BatchNorm partials of the stored output: per column, per group slot {sum, M2}
  if (d->stat_part) {
    const int gr = d->stat_gr;
    const int trow0 = tm * BM;
    const int gfirst = trow0 / gr;
    const int gsplit = (gfirst + 1) * gr;   // first row of slot 1 (a tile spans <= 2 groups)
    float part[2][2];
    for (int s = 0; s < 2; ++s) {
      // pass 1: sum
      float sum = 0.f;
      if (owner && colok) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = rbase + (r & 3) + 8 * (r >> 2);
          if (row < M && (row >= gsplit) == (s == 1)) sum += v[r];
        }
      }
      sum += __shfl_xor(sum, 32);
      if (owner && lh == 0) s_col[(wm * WN + wn) * 32 + li] = sum;
      __syncthreads();
      float tot = 0.f;
      for (int q = 0; q < WM; ++q) tot += s_col[(q * WN + wn) * 32 + li];
      __syncthreads();
      const int ra = max(trow0, (gfirst + s) * gr), rb = min(min(trow0 + BM, M), (gfirst + s + 1) * gr);
      const int cnt = rb - ra;
      const float mean = cnt > 0 ? tot / cnt : 0.f;
      // pass 2: M2 about the tile-slot mean
      float q2 = 0.f;
      if (owner && colok) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = rbase + (r & 3) + 8 * (r >> 2);
          if (row < M && (row >= gsplit) == (s == 1)) {
            const float dd = v[r] - mean;
            q2 += dd * dd;
          }
        }
      }
      q2 += __shfl_xor(q2, 32);
      if (owner && lh == 0) s_col[(wm * WN + wn) * 32 + li] = q2;
      __syncthreads();
      float qt = 0.f;
      for (int q = 0; q < WM; ++q) qt += s_col[(q * WN + wn) * 32 + li];
      __syncthreads();
      part[s][0] = cnt > 0 ? tot : 0.f;
      part[s][1] = cnt > 0 ? qt : 0.f;
    }
    if (owner && wm == 0 && lh == 0 && colok) {
      for (int s = 0; s < 2; ++s) {
        float* p = d->stat_part + ((long)(tm * 2 + s) * N + col) * 2;
        gst(p, part[s][0]);
        gst(p + 1, part[s][1]);
      }
    }
  }

  if (owner && colok) {
    if (ones_col) {
      if (d->bias_out) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = rbase + (r & 3) + 8 * (r >> 2);
          if (row < M) gst(d->bias_out + row, v[r]);
        }
      }
    } else {
      float* __restrict__ C = d->C;
      const int ldc = d->ldc;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rbase + (r & 3) + 8 * (r >> 2);
        if (row < M) gst(C + (long)row * ldc + col, v[r]);
      }
    }
  }
}

// One kernel symbol for every GEMM of the step; a grouped launch may mix layouts (e.g. the
// weight gradient (TN) and the input gradient (NN) of one layer run side by side).
// Dynamic LDS: [tf_floats: BatchNorm scale/shift table (0 when no problem of the launch needs it)]
//              [staging slices of every k-group, reused for the split-K partials after the loop]
__global__ __launch_bounds__(CGL_GEMM_THREADS) void cgl_gemm_f32(const CglGemmDesc* __restrict__ descs, int ndesc,
                                                                 int tf_floats) {
  extern __shared__ float cgl_dyn_lds[];
  __shared__ float s_col[4 * 32 * 2];           // per-column reductions across waves
  float* s_tf = cgl_dyn_lds;
  float* s_stage = cgl_dyn_lds + tf_floats;
  const int bid = blockIdx.x;
  int di = 0;
  for (int q = 1; q < ndesc; ++q)
    if (bid >= descs[q].wg_begin) di = q;
  const CglGemmDesc* __restrict__ d = descs + di;
  const int layout = d->layout;
  // VEC: every operand allows 16-byte loads along its contiguous dimension
  const int vec = d->a_vec && d->b_vec;
  const int pipe = d->pipe;
#define CGL_BODY(L)                                             \
  do {                                                          \
    if (pipe) {                                                 \
      if (vec)                                                  \
        cgl_gemm_body<L, 1, 1>(d, bid, s_tf, s_stage, s_col);   \
      else                                                      \
        cgl_gemm_body<L, 0, 1>(d, bid, s_tf, s_stage, s_col);   \
    } else {                                                    \
      if (vec)                                                  \
        cgl_gemm_body<L, 1, 0>(d, bid, s_tf, s_stage, s_col);   \
      else                                                      \
        cgl_gemm_body<L, 0, 0>(d, bid, s_tf, s_stage, s_col);   \
    }                                                           \
  } while (0)
  if (layout == 0)
    CGL_BODY(0);
  else if (layout == 1)
    CGL_BODY(1);
  else
    CGL_BODY(2);
#undef CGL_BODY
}

// Host helper: dynamic LDS bytes of one problem (staging or split-K region; the table is extra).
inline int cgl_gemm_stage_bytes(const CglGemmDesc& d) {
  const int red = 3 * 16 * 64 * 4;
  const int st = d.pipe ? d.WK * 2 * (32 * d.WM + 32 * d.WN) * CGL_LDK * 4 : 0;
  return st > red ? st : red;
}
