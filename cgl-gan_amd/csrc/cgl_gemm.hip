// fp32 MFMA GEMM for the MLP GAN step (gfx950, v_mfma_f32_32x32x2_f32).
//
// Replaces the reference's implicit cuBLAS addmm / mm calls of nn.Linear forward and
// autograd backward (model/mnist_model.py:11,22,77,79,81), with the
// BatchNorm1d(train) + LeakyReLU of model/mnist_model.py:13-14 folded into the operand loads.
//
// Design (MI355X-first, not a CUDA tiling):
//  * one wave owns TM x TN 32x32 f32 MFMA accumulators (1x1 for small problems, 2x2 for the
//    large ones); v_mfma_f32_32x32x2_f32 issues every 64 cycles with a 64-cycle dependent
//    latency, so even a single accumulation chain runs at the f32 matrix peak;
//  * a 256-thread workgroup holds 4 waves arranged WM x WN x WK: WK > 1 splits K inside the
//    workgroup (skinny, batch-256 GEMMs need it to put >= 1024 waves on the 256 CUs) and the
//    split is summed through LDS in a fixed order (deterministic, no atomics);
//  * operands are loaded straight into the MFMA fragment registers.  The k index of the
//    32x32x2 fragment is permuted so that lane half h owns 8 CONSECUTIVE k of every 16-k
//    chunk: a k-contiguous operand is then two float4 loads per lane per 8 MFMAs;
//  * A-operand transforms applied between the load and the MFMA (no separate launch):
//      a_bn 1  BatchNorm1d(train) + LeakyReLU of a k-contiguous A (the previous layer's Linear
//              output): the workgroup prologue combines the producer GEMM's per-tile {sum, M2}
//              partials of the forward call its rows belong to into scale / shift per k (LDS);
//              workgroup 0 also writes the saved mean / invstd and the running statistics;
//      a_bn 2  BatchNorm1d backward of A = dy (the LeakyReLU'-masked gradient the previous GEMM
//              stored with its {sum dy, sum (y - mean) dy} partials): dZ = (dy - S/M - (y - mean)
//              D invstd^2 / M) invstd gamma per k (k-contiguous A) or per m (m-contiguous A),
//              the BatchNorm input y streamed beside A; workgroup 0 writes dgamma / dbeta;
//  * prologue fusion: the A operand rows can be gathered through an index list (the sampled
//    real batch) from two sources (real rows, then generated rows) and written out once
//    (the copy-out of each 16-k chunk is spread over the workgroups that load it);
//  * epilogue fusion: bias, LeakyReLU / Tanh, LeakyReLU' mask, Tanh' (1 - t^2), the
//    bias-gradient column (B's extra all-ones column), per-column {sum, M2} partials of the
//    stored output for the next layer's forward BatchNorm, and per-column {sum dy,
//    sum (y - mean) dy} partials of the stored gradient for its backward BatchNorm.
#include "cgl_internal.h"

#include <type_traits>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// 16-bit operand GEMMs (cgl_gan_config.gemm_dtype, BASELINE config 5): the fp32 operands are
// rounded to fp16 / bf16 (round-to-nearest-even) as they enter the MFMA; products are exact and
// accumulate in fp32.  The k-permuted fragment of a 16-k chunk (lane half h holds k = 8h .. 8h + 7)
// is exactly the operand of v_mfma_f32_32x32x16_{f16,bf16}, so one MFMA replaces the eight
// 32x32x2 f32 MFMAs of the chunk.
template <int DT>
__device__ __forceinline__ void cgl_mfma16(f32x16& acc, const float (&a)[8], const float (&b)[8]) {
  if constexpr (DT == CGL_DTYPE_F16) {
    f16x8 x, y;
#pragma unroll
    for (int q = 0; q < 8; ++q) { x[q] = (_Float16)a[q]; y[q] = (_Float16)b[q]; }
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(x, y, acc, 0, 0, 0);
  } else {
    bf16x8 x, y;
#pragma unroll
    for (int q = 0; q < 8; ++q) { x[q] = (__bf16)a[q]; y[q] = (__bf16)b[q]; }
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, y, acc, 0, 0, 0);
  }
}

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

// ------------------------------------------------------------------------------------------
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

// a_bn 1 prologue: scale / shift of every k of this workgroup's forward call g into the LDS
// tables t_sc / t_sh (torch's arithmetic: invstd = 1 / sqrt(var_biased + eps), scale = invstd
// gamma, shift = beta - mean scale); workgroup 0 (lead) combines every call -- in the reference's
// call order (Xd then Xg) -- to write the saved mean / invstd and update the running statistics.
__device__ __forceinline__ void cgl_abn_fwd_prologue(const CglBnFwd& bn, int K, int g, bool lead, float* t_sc,
                                                     float* t_sh) {
  // every {sum, M2} pair this thread needs (Q features x <= 8 tiles) is loaded at once: one memory
  // round trip per forward call (the register peak is here, not in the main loop)
  const int tid = threadIdx.x;
  const int ng = (bn.mtot + bn.gr - 1) / bn.gr;     // <= 2 (planner)
  constexpr int Q = CGL_BN_MAXF / 256;
  int k[Q];
  float rm[Q], rv[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    k[q] = tid + 256 * q < K ? tid + 256 * q : -1;
    rm[q] = rv[q] = 0.f;
  }
  if (lead && bn.run_mean) {
#pragma unroll
    for (int q = 0; q < Q; ++q)
      if (k[q] >= 0) {
        rm[q] = gld(bn.run_mean + k[q]);
        rv[q] = gld(bn.run_var + k[q]);
      }
  }
  for (int gg = 0; gg < ng; ++gg) {
    if (!lead && gg != g) continue;
    double mean[Q], m2[Q];
    int n;
    cgl_bn_stats<Q>(bn, K, k, gg, mean, m2, n);
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      if (k[q] < 0) continue;
      const double invstd = 1.0 / sqrt(m2[q] / n + bn.eps);
      if (gg == g) {
        const float sc = (float)invstd * gld(bn.gamma + k[q]);
        t_sc[k[q]] = sc;
        t_sh[k[q]] = gld(bn.beta + k[q]) - (float)mean[q] * sc;
      }
      if (lead) {
        if (bn.save_mean) {
          gst(bn.save_mean + (long)gg * K + k[q], (float)mean[q]);
          gst(bn.save_invstd + (long)gg * K + k[q], (float)invstd);
        }
        if (bn.run_mean) {
          const double mom = bn.momentum;
          rm[q] = (float)(mom * mean[q] + (1.0 - mom) * (double)rm[q]);
          rv[q] = (float)(mom * (m2[q] / (n - 1)) + (1.0 - mom) * (double)rv[q]);
        }
      }
    }
  }
  if (lead && bn.run_mean) {
#pragma unroll
    for (int q = 0; q < Q; ++q)
      if (k[q] >= 0) {
        gst(bn.run_mean + k[q], rm[q]);
        gst(bn.run_var + k[q], rv[q]);
      }
  }
}

// a_bn 2 prologue: per feature f in [f0, f1) the backward coefficients of torch's
// batch_norm_backward (train) from the producer's per-row-tile {sum dy, sum (y - mean) dy}
// partials (tile order, double): mean, invstd, gamma, S / M, D invstd^2 / M (as cgl_bn_bwd
// computes them, in float); lead: dgamma = D invstd, dbeta = S.
__device__ __forceinline__ void cgl_abn_bwd_prologue(const CglBnBwdFold& b, int f0, int f1, bool lead, float* t) {
  typedef double f64x2 __attribute__((ext_vector_type(2)));
  const int tid = threadIdx.x;
  for (int f = f0 + tid; f < f1; f += 256) {
    // the tiles' partials in groups of 8 loads in flight, summed in tile order
    double S = 0.0, D = 0.0;
    for (int t0 = 0; t0 < b.tiles; t0 += 8) {
      f64x2 pr[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        pr[j] = *(const CGL_GLOBAL f64x2*)(b.part + ((long)min(t0 + j, b.tiles - 1) * b.F + f) * 2);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (t0 + j < b.tiles) {
          S += pr[j][0];
          D += pr[j][1];
        }
    }
    const float invstd = gld(b.invstd + f);
    const int i = f - f0;
    t[0 * CGL_BNB_TAB + i] = gld(b.mean + f);
    t[1 * CGL_BNB_TAB + i] = invstd;
    t[2 * CGL_BNB_TAB + i] = gld(b.gamma + f);
    t[3 * CGL_BNB_TAB + i] = (float)(S / b.M);
    t[4 * CGL_BNB_TAB + i] = (float)D * invstd * invstd / b.M;
    if (lead) {
      gst(b.g_gamma + f, (float)(D * (double)invstd));
      gst(b.g_beta + f, (float)S);
    }
  }
}

// dZ of one element: torch's (dy - S/M - (y - mean) D invstd^2 / M) invstd gamma, as cgl_bn_bwd
__device__ __forceinline__ float cgl_bnb_apply(float dy, float y, float mean, float invstd, float w, float gm, float kk) {
  return (dy - gm - (y - mean) * kk) * invstd * w;
}

// Epilogue Adam of one accumulator block's 16 gradient values (rows rb + (r & 3) + 8 (r >> 2), column col
// of a row-major [M][ld] tensor): all parameter / moment loads issued first, then cgl_adam_update -- the
// arithmetic of cgl_adam on the same gradient values, so the result is bitwise cgl_adam's.
__device__ __forceinline__ void cgl_epi_adam(const CglGemmDesc* __restrict__ d, float* p_, float* m_, float* v_,
                                             int rb, int M, int col, int ld, const float* g) {
  const float ss = gld(d->ad_ss), bc = gld(d->ad_bc);
  float p[16], m[16], v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const long e = (long)min(rb + (r & 3) + 8 * (r >> 2), M - 1) * ld + col;
    p[r] = gld(p_ + e);
    m[r] = gld(m_ + e);
    v[r] = gld(v_ + e);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = rb + (r & 3) + 8 * (r >> 2);
    cgl_adam_update(p[r], g[r], m[r], v[r], ss, bc, d->ad_b2, d->ad_w1, d->ad_w2, d->ad_eps);
    if (row < M) {
      const long e = (long)row * ld + col;
      gst(m_ + e, m[r]);
      gst(v_ + e, v[r]);
      gst(p_ + e, p[r]);
    }
  }
}

// ------------------------------------------------------------------------------------------
// Main body.  One wave owns TM x TN 32x32 accumulator blocks ((32 TM) x (32 TN) outputs); the
// workgroup tile is (32 TM WM) x (32 TN WN), K split WK ways.  Operand fragments of S chunks
// (16 k each) are in flight in a rotation of S register sets, so (S - 1) x TM TN x 512 MFMA
// cycles cover an L2 / MALL miss; TM = TN = 2 halves the operand traffic per FLOP and
// quadruples the MFMA work per load batch for the large problems.
template <int TM, int TN>
struct CglPipe {
#ifndef CGL_GEMM_STAGES
#define CGL_GEMM_STAGES 3
#endif
#ifndef CGL_GEMM_STAGES1
#define CGL_GEMM_STAGES1 CGL_GEMM_STAGES
#endif
  // 1x1-block waves (16 staging floats per chunk) can afford a deeper rotation than 2x2 ones
  static constexpr int S = (TM * TN == 1) ? CGL_GEMM_STAGES1 : CGL_GEMM_STAGES;
};

// Compile-time flags of a main-loop version: packed A, packed B (layout 0 only), A copy-out.
template <bool A_, bool B_, bool C_>
struct CglLoopFl {
  static constexpr bool PA = A_, PB = B_, CP = C_;
};

// Dynamic LDS layout: [operand-transform tables (cgl_gemm_tab_floats)] [split-K partials]
template <int LAYOUT, int VEC, int TM, int TN, bool SK, int DT = 0, int ABN = 0, bool ADAM = false>
__device__ __forceinline__ void cgl_gemm_body(const CglGemmDesc* __restrict__ d, int bid, float* __restrict__ s_dyn,
                                              int* __restrict__ s_flag,
                                              double* __restrict__ s_bnd, unsigned long long t_entry = 0) {
  constexpr int S = CglPipe<TM, TN>::S;
  // The descriptor fields the set-up and the k-loop prologue need, read in ONE round of scalar loads before the
  // first branch and pinned there: left to the compiler, each load is issued in the block that uses it, after
  // that block's branch -- a chain of dependent scalar round trips (~0.16 us each, tools/launch_probe.hip) at
  // every launch start (tools/gemm_trace.py: ~1.7 us from kernel entry to the k-loop in the round 4 build).
  const int M = d->M, N = d->N, K = d->K;
  const int WN = d->WN, WK = d->WK, WM = d->WM;
  const int h_tm = d->tiles_m, h_tn = d->tiles_n, h_wg0 = d->wg_begin, h_ks = SK ? d->ksplit : 1;
  const int h_xcd = d->xcd_pm, h_tab = d->tab_floats, h_gen = d->a_gen, h_abn = ABN ? d->a_bn : 0;
  const int h_ones = (LAYOUT != 0) ? d->b_ones_col : 0, h_apk = d->a_pk, h_bpk = d->b_pk;
  const float* const h_bias = d->bias;
  const float* const h_mref = d->mask_ref;
  const float* const h_tref = d->tanh_ref;
  const int h_mld = d->mask_ld, h_tld = d->tanh_ld, h_crow0 = d->a_copy_row0;
  float* const h_copy = d->a_copy;
  const CglRowSrc h_a = d->a, h_b = d->b;
  // the epilogue's fields too (they would otherwise cost one more scalar round trip after the k-loop)
  const int e_act = d->act, e_ldc = d->ldc, e_gr = d->stat_gr;
#ifndef CGL_GEMM_NO_CPERM
  const int e_cperm = d->c_perm;
#else
  const int e_cperm = 0;     // (A/B builds: the output-row permutation compiled out)
#endif
  const float e_slope = d->slope;
  float* const e_C = d->C;
  float* const e_bout = d->bias_out;
  float* const e_stat = d->stat_part;
  double* const e_bnb = d->bnb_part;
  // every read above issued before anything uses one of them: ONE batch of scalar loads and one wait (left to
  // itself the scheduler started the tile arithmetic on the first batch and waited a second time)
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::"s"(M), "s"(N), "s"(K), "s"(WN), "s"(WK), "s"(WM), "s"(h_tm), "s"(h_tn), "s"(h_wg0), "s"(h_ks),
               "s"(h_xcd), "s"(h_tab), "s"(h_gen), "s"(h_abn), "s"(h_ones), "s"(h_apk), "s"(h_bpk));
  asm volatile("" ::"s"(e_act), "s"(e_ldc), "s"(e_gr), "s"(e_slope), "s"(e_C), "s"(e_bout), "s"(e_stat), "s"(e_bnb),
               "s"(e_cperm));
  asm volatile("" ::"s"(h_bias), "s"(h_mref), "s"(h_tref), "s"(h_mld), "s"(h_tld), "s"(h_crow0), "s"(h_copy),
               "s"(h_a.p0), "s"(h_a.p1), "s"(h_a.idx0), "s"(h_a.idx_off), "s"(h_a.split), "s"(h_a.ld), "s"(h_b.p0),
               "s"(h_b.p1), "s"(h_b.idx0), "s"(h_b.idx_off), "s"(h_b.split), "s"(h_b.ld));
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int li = lane & 31, lh = lane >> 5;
  const int wk = wave % WK, wmn = wave / WK;
  const int wm = wmn / WN, wn = wmn % WN;
  // XCD-aware tile order (blocks b and b+8 land on the same XCD): each XCD takes a contiguous
  // range of (tile, k-slice) units in n-major order, so its L2 holds ~1/8 of the B panels (the
  // weights) plus the A panels, instead of all of both, and the k-slices of one tile share an XCD
  // (their partials stay XCD-local).  Bijective for any count (guide T1).
  const int KS = (SK && h_ks > 1) ? h_ks : 1;   // SK: the split-K instantiation
  const int local = bid - h_wg0;
  const int ntile = h_tm * h_tn;
  const int nwg = ntile * KS;
  int unit = local;
  if (nwg >= 16) {
    const int xcd = local & 7, pos = local >> 3, q = nwg >> 3, r = nwg & 7;
    unit = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
  }
  int tile = unit / KS;
  const int kslice = unit - tile * KS;
  int tn, tm;
  if (h_xcd > 0 && nwg >= 16) {
    // XCD blocking: position `tile` of the XCD-contiguous sequence is tile `tile` of the slab-major order --
    // slab x = (row slab x / pn, column slab x % pn) of a pm x pn cut of the tile grid, tiles m-minor inside
    // a slab -- so the XCD running a range of the sequence reads one row slab of A and one column slab of B
    // instead of all of A (the n-major order) or all of B.  Bijective for any grid.
    const int pm = h_xcd, pn = 8 / pm, TMt = h_tm, TNt = h_tn;
    int rest = tile, x = 0, r0 = 0, r1 = 0, c0 = 0, c1 = 0;
    for (; x < 8; ++x) {
      r0 = (x / pn) * TMt / pm;
      r1 = (x / pn + 1) * TMt / pm;
      c0 = (x % pn) * TNt / pn;
      c1 = (x % pn + 1) * TNt / pn;
      const int sz = (r1 - r0) * (c1 - c0);
      if (rest < sz) break;
      rest -= sz;
    }
    const int h = r1 - r0;
    tn = c0 + rest / h;
    tm = r0 + rest % h;
    tile = tn * TMt + tm;
  } else {
    tn = tile / h_tm;
    tm = tile % h_tm;
  }
#ifdef CGL_GEMM_TRACE
  unsigned long long* trc = (d->trace && local < CGL_GEMM_TRACE_WGS) ? d->trace + (long)local * CGL_GEMM_TRACE_W : nullptr;
  if (trc && tid == 0) {
    trc[0] = t_entry;
    trc[1] = wall_clock64();
  }
#endif
  const int BM = 32 * TM * WM;
  const int m0 = tm * BM + wm * 32 * TM;            // first row of this wave's tile
  const int n0 = (tn * WN + wn) * 32 * TN;          // first column of this wave's tile
  float* __restrict__ s_tab = s_dyn;                // operand-transform tables
  float* __restrict__ s_red = s_dyn + h_tab;   // split-K partials

  // ---------------- generated A rows (the fused round prologue): this tile's rows of z, drawn here
  if (h_gen) {
    const int r0 = tm * BM, r1 = min(r0 + BM, M);
    const long q0 = ((long)r0 * K) >> 2, q1 = ((long)r1 * K + 3) >> 2;
    const uint32_t rnd = (uint32_t)(gldi(d->gen_round) + 1);
    for (long q = q0 + tid; q < q1; q += CGL_GEMM_THREADS)
      cgl_normal_at(q, const_cast<float*>(h_a.p0), d->gen_n, d->gen_seed, rnd, 0);
    __syncthreads();   // (workgroup release / acquire: the rows are read back below, by every wave)
  }

  // ---------------- operand-transform prologue (before any operand load is consumed)
  // ABN: the instantiation carrying the operand transforms (0: none compiled in; 1 / 2: the mode
  // of the launch's problems, a problem with a_bn 0 beside them runs untransformed)
  const int abn = h_abn;
  if (ABN == 1 && abn == 1) {                 // forward BatchNorm of A (k-contiguous, every k)
    cgl_abn_fwd_prologue(d->a_bnf, K, (tm * BM) / d->a_bnf.gr, local == 0 && kslice == 0, s_tab,
                         s_tab + CGL_BN_MAXF + 16);
    __syncthreads();
  } else if (ABN == 2 && abn == 2) {   // backward BatchNorm of A: every k (kc) or this tile's m range (mn)
    const int f0 = LAYOUT == 2 ? tm * BM : 0, f1 = LAYOUT == 2 ? min(tm * BM + BM, M) : K;
    cgl_abn_bwd_prologue(d->a_bnb, f0, f1, LAYOUT != 2 && local == 0 && kslice == 0, s_tab);
    __syncthreads();
  }
  // per-lane coefficients of an m-contiguous A under a_bn 2 (its lane's row m is fixed)
  float bm_mean[TM], bm_inv[TM], bm_w[TM], bm_gm[TM], bm_k[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    bm_mean[i] = bm_inv[i] = bm_w[i] = bm_gm[i] = bm_k[i] = 0.f;
    if (ABN == 2 && LAYOUT == 2 && abn == 2) {
      const int r = min(m0 + 32 * i + li, M - 1) - tm * BM;
      bm_mean[i] = s_tab[0 * CGL_BNB_TAB + r];
      bm_inv[i] = s_tab[1 * CGL_BNB_TAB + r];
      bm_w[i] = s_tab[2 * CGL_BNB_TAB + r];
      bm_gm[i] = s_tab[3 * CGL_BNB_TAB + r];
      bm_k[i] = s_tab[4 * CGL_BNB_TAB + r];
    }
  }

  // ---------------- epilogue operands, issued before the k-loop
  // The bias and the LeakyReLU' / Tanh' reference of the stored tile are loaded by the owner waves
  // ahead of the first chunk's operands: they return with that chunk (loads count in order) instead
  // of costing one more dependent memory round trip after the k-loop.  (A descriptor carries at most
  // one of mask_ref / tanh_ref.)  Clamped addresses, unconditional per lane.  CGL_GEMM_EPI_PF=0 keeps the
  // loads in the epilogue.
#ifndef CGL_GEMM_EPI_PF
#define CGL_GEMM_EPI_PF 1
#endif
  constexpr bool EPF = CGL_GEMM_EPI_PF && !ADAM && TM * TN == 1;   // (2x2 waves: no registers to spare)
  float pf_bias[TN], pf_ref[EPF ? TM : 1][EPF ? TN : 1][16];
  if constexpr (EPF) {
    if (wk == 0) {
      const float* ref = h_mref ? h_mref : h_tref;
      const long ldr = h_mref ? h_mld : h_tld;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int colc = min(n0 + 32 * j + li, N - 1);
        pf_bias[j] = h_bias ? gld(h_bias + colc) : 0.f;
        if (ref) {
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int row = min(m0 + 4 * lh + 32 * i + (r & 3) + 8 * (r >> 2), M - 1);
              pf_ref[i][j][r] = gld(ref + (long)row * ldr + colc);
            }
        }
      }
    }
  }

  // ---------------- main loop
  const int b_ones = h_ones;
  const int nmem = N - b_ones;     // columns of B actually in memory
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
#ifndef CGL_GEMM_NACC
#define CGL_GEMM_NACC 2
#endif
  // 1x1 blocks: NACC independent accumulation chains over alternating k-steps of a chunk (summed in
  // a fixed order after the k-loop), so consecutive MFMAs do not wait on each other's result
  constexpr int NX = (TM * TN == 1 && DT == CGL_DTYPE_F32) ? CGL_GEMM_NACC : 1;
  f32x16 accx[NX > 1 ? NX - 1 : 1];
#pragma unroll
  for (int x = 0; x < (NX > 1 ? NX - 1 : 1); ++x)
#pragma unroll
    for (int r = 0; r < 16; ++r) accx[x][r] = 0.f;

#ifdef CGL_GEMM_TRACE
  if (trc && tid == 0) trc[2] = wall_clock64();
#endif
  {
  const int nch = (K + CGL_GEMM_KCHUNK - 1) / CGL_GEMM_KCHUNK;
  // chunk range of this wave: slice kslice * WK + wk of KS * WK equal slices of the K chunks
  const int nsl = KS * WK, sl = kslice * WK + wk;
  const int cb = (sl * nch) / nsl, ce = ((sl + 1) * nch) / nsl;
  const int lda = h_a.ld, ldb = h_b.ld;
  float* __restrict__ a_copy = h_copy;
  // copy-out: chunk c of a row block is written by the one wave of the (tiles_n x WN) that load
  // it whose column index equals c modulo their count (the copy work spread over every workgroup)
  const int copy_n = h_tn * WN, copy_me = tn * WN + wn;
  const bool ybn = ABN == 2 && abn == 2;        // A under a_bn 2 streams the BatchNorm input y
  const float* __restrict__ ybase = d->a_bnb.y;
  const int ldy = d->a_bnb.ldy;

  // per-lane operand rows / columns of each block, clamped (always dereferenceable) bases
  const float* a_base[TM];
  const float* y_base[TM];
  const float* b_base[TN];
  bool b_is_ones[TN], copy_row[TM];
  const int kcn = (K + CGL_GEMM_KCHUNK - 1) / CGL_GEMM_KCHUNK;   // k chunks (packed block stride)
  const bool apk = LAYOUT == 0 && h_apk, bpk = LAYOUT == 0 && h_bpk;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int am = m0 + 32 * i + li;      // A row (kc) or A column (mn)
    a_base[i] = (LAYOUT != 2) ? cgl_row(h_a, min(am, M - 1)) : h_a.p0 + min(am, M - 1);
    // packed A: the lane's float4 of chunk 0 of its (clamped) 32-row block
    if (apk) a_base[i] = h_a.p0 + (long)(min(m0 + 32 * i, (M - 1) & ~31) >> 5) * kcn * 512 + lane * 4;
    y_base[i] = ybn ? ((LAYOUT != 2) ? ybase + (long)min(am, M - 1) * ldy : ybase + min(am, M - 1)) : a_base[i];
    copy_row[i] = (LAYOUT != 2) && a_copy && am < M && am >= h_crow0;
  }
  // A copy-out in the main loop (full chunks, 16-byte form) as buffer stores whose offset is pushed out of range
  // for the lanes / chunks that do not write: no branch in the loop body, so every s_waitcnt there still counts
  // exactly the loads of the set it consumes (a conditional store made the compiler drain vmcnt(0) at the top of
  // every rotation).  The range check drops the out-of-range stores.
  const auto rc_copy = __builtin_amdgcn_make_buffer_rsrc(a_copy ? a_copy : const_cast<float*>(h_a.p0), (short)0,
                                                         0x7fffffff, 0x00020000);
  unsigned copy_off[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i)
    copy_off[i] = copy_row[i] ? (unsigned)((m0 + 32 * i + li) * d->a_copy_ld) * 4u : 0x7fffffffu;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int bc = n0 + 32 * j + li;      // B row (NT) or B column (NN/TN)
    b_is_ones[j] = b_ones && (bc == N - 1);
    b_base[j] = (LAYOUT == 0) ? cgl_row(h_b, min(bc, N - 1)) : h_b.p0 + max(0, min(bc, nmem - 1));
    if (bpk) b_base[j] = h_b.p0 + (long)(min(n0 + 32 * j, (N - 1) & ~31) >> 5) * kcn * 512 + lane * 4;
  }

  // Full chunks (k + 16 <= K) load without clamps and multiply without masks: rows / columns
  // past M / N come from clamped (valid) addresses and only feed accumulator rows / columns
  // that are never stored.  Only the K-tail chunk clamps its k and zeroes k >= K.
  auto load_a = [&](auto tail, int c, const float* const (&base)[TM], int ld, float (&A_)[TM][8], auto pkc) {
    constexpr bool T = decltype(tail)::value;
    constexpr bool pk = decltype(pkc)::value;
    const int k = c * CGL_GEMM_KCHUNK + 8 * lh;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      if constexpr (LAYOUT == 0 && pk) {          // packed: two contiguous 1 KB wave loads (padding past K)
        const f32x4 x = *(gcf4p)(base[i] + c * 512), y = *(gcf4p)(base[i] + c * 512 + 256);
        A_[i][0] = x[0]; A_[i][1] = x[1]; A_[i][2] = x[2]; A_[i][3] = x[3];
        A_[i][4] = y[0]; A_[i][5] = y[1]; A_[i][6] = y[2]; A_[i][7] = y[3];
      } else if (LAYOUT == 2) {
        if (T) {
          cgl_ld_mn(base[i], ld, k, K, A_[i]);
        } else {
          gcfp q = (gcfp)base[i] + (long)k * ld;
#pragma unroll
          for (int j = 0; j < 8; ++j) A_[i][j] = q[(long)j * ld];
        }
      } else {
        if (T) {
          cgl_ld_kc<VEC>(base[i], k, K, A_[i]);
        } else if (VEC) {
          const f32x4 x = *(gcf4p)(base[i] + k), y = *(gcf4p)(base[i] + k + 4);
          A_[i][0] = x[0]; A_[i][1] = x[1]; A_[i][2] = x[2]; A_[i][3] = x[3];
          A_[i][4] = y[0]; A_[i][5] = y[1]; A_[i][6] = y[2]; A_[i][7] = y[3];
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) A_[i][j] = ((gcfp)base[i])[k + j];
        }
      }
    }
  };
  // fl: the loop version's compile-time flags (LoopFl: packed A, packed B, copy-out) -- see run_loop below
  auto load_chunk = [&](auto tail, int c, float (&A_)[TM][8], auto& Y_, float (&B_)[TN][8], auto fl) {
    constexpr bool T = decltype(tail)::value;
    const int k = c * CGL_GEMM_KCHUNK + 8 * lh;
    load_a(tail, c, a_base, lda, A_, std::integral_constant<bool, decltype(fl)::PA>());
    if constexpr (ABN == 2)
      if (ybn) load_a(tail, c, y_base, ldy, Y_, std::integral_constant<bool, false>());
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if constexpr (LAYOUT == 0 && decltype(fl)::PB) {
        const f32x4 x = *(gcf4p)(b_base[j] + c * 512), y = *(gcf4p)(b_base[j] + c * 512 + 256);
        B_[j][0] = x[0]; B_[j][1] = x[1]; B_[j][2] = x[2]; B_[j][3] = x[3];
        B_[j][4] = y[0]; B_[j][5] = y[1]; B_[j][6] = y[2]; B_[j][7] = y[3];
      } else if (LAYOUT == 0) {
        if (T) {
          cgl_ld_kc<VEC>(b_base[j], k, K, B_[j]);
        } else if (VEC) {
          const f32x4 x = *(gcf4p)(b_base[j] + k), y = *(gcf4p)(b_base[j] + k + 4);
          B_[j][0] = x[0]; B_[j][1] = x[1]; B_[j][2] = x[2]; B_[j][3] = x[3];
          B_[j][4] = y[0]; B_[j][5] = y[1]; B_[j][6] = y[2]; B_[j][7] = y[3];
        } else {
#pragma unroll
          for (int q = 0; q < 8; ++q) B_[j][q] = ((gcfp)b_base[j])[k + q];
        }
      } else {
        if (T) {
          cgl_ld_mn(b_base[j], ldb, k, K, B_[j]);
        } else {
          gcfp q = (gcfp)b_base[j] + (long)k * ldb;
#pragma unroll
          for (int u = 0; u < 8; ++u) B_[j][u] = q[(long)u * ldb];
        }
      }
    }
  };
  auto compute_chunk = [&](auto tail, int c, float (&A_)[TM][8], auto& Y_, float (&B_)[TN][8], auto fl) {
    constexpr bool T = decltype(tail)::value;
    const int k = c * CGL_GEMM_KCHUNK + 8 * lh;
    if (ABN == 1 && abn == 1 && LAYOUT == 0) {
      // BatchNorm1d(train) + LeakyReLU of the Linear output, scale / shift of k from LDS
      // (the 8 k of a lane half are contiguous: two 16-byte LDS reads per table)
      const f32x4 sc0 = *(const f32x4*)(s_tab + k), sc1 = *(const f32x4*)(s_tab + k + 4);
      const f32x4 sh0 = *(const f32x4*)(s_tab + CGL_BN_MAXF + 16 + k);
      const f32x4 sh1 = *(const f32x4*)(s_tab + CGL_BN_MAXF + 16 + k + 4);
      const float sc[8] = {sc0[0], sc0[1], sc0[2], sc0[3], sc1[0], sc1[1], sc1[2], sc1[3]};
      const float sh[8] = {sh0[0], sh0[1], sh0[2], sh0[3], sh1[0], sh1[1], sh1[2], sh1[3]};
      const float sl = d->a_bnf.slope;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float x = fmaf(A_[i][q], sc[q], sh[q]);
          A_[i][q] = x > 0.f ? x : x * sl;
        }
    } else if constexpr (ABN == 2) {
     if (abn == 2) {
      if (LAYOUT == 2) {       // m-contiguous A: the lane's feature is fixed
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int q = 0; q < 8; ++q)
            A_[i][q] = cgl_bnb_apply(A_[i][q], Y_[i][q], bm_mean[i], bm_inv[i], bm_w[i], bm_gm[i], bm_k[i]);
      } else {                 // k-contiguous A: the 8 k of the lane half (two 16-byte LDS reads
        float cf[5][8];        // per table; past K in the tail chunk: padding, masked below)
#pragma unroll
        for (int t = 0; t < 5; ++t) {
          const f32x4 u0 = *(const f32x4*)(s_tab + t * CGL_BNB_TAB + k);
          const f32x4 u1 = *(const f32x4*)(s_tab + t * CGL_BNB_TAB + k + 4);
          cf[t][0] = u0[0]; cf[t][1] = u0[1]; cf[t][2] = u0[2]; cf[t][3] = u0[3];
          cf[t][4] = u1[0]; cf[t][5] = u1[1]; cf[t][6] = u1[2]; cf[t][7] = u1[3];
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int q = 0; q < 8; ++q)
            A_[i][q] = cgl_bnb_apply(A_[i][q], Y_[i][q], cf[0][q], cf[1][q], cf[2][q], cf[3][q], cf[4][q]);
      }
     }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      if (T) cgl_mask(A_[i], true, k, K);
      if constexpr (!decltype(fl)::CP) continue;
      if (VEC && !T) {
        const unsigned off = (c % copy_n) == copy_me ? copy_off[i] + 4u * k : 0x7fffffffu;
        __builtin_amdgcn_raw_buffer_store_b128(f32x4{A_[i][0], A_[i][1], A_[i][2], A_[i][3]}, rc_copy, off, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(f32x4{A_[i][4], A_[i][5], A_[i][6], A_[i][7]}, rc_copy, off + 16u, 0, 0);
      } else if (copy_row[i] && (c % copy_n) == copy_me) {
        float* dst = a_copy + (long)(m0 + 32 * i + li) * d->a_copy_ld;
        if (VEC && (!T || k + 7 < K)) {
          *(gf4p)(dst + k) = f32x4{A_[i][0], A_[i][1], A_[i][2], A_[i][3]};
          *(gf4p)(dst + k + 4) = f32x4{A_[i][4], A_[i][5], A_[i][6], A_[i][7]};
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (!T || k + j < K) gst(dst + k + j, A_[i][j]);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if (T) cgl_mask(B_[j], true, k, K);
      if (b_ones) {
#pragma unroll
        for (int q = 0; q < 8; ++q)
          if (b_is_ones[j]) B_[j][q] = (!T || k + q < K) ? 1.f : 0.f;
      }
    }
    if constexpr (DT != CGL_DTYPE_F32) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) cgl_mfma16<DT>(acc[i][j], A_[i], B_[j]);
    } else if constexpr (NX > 1) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        if (q % NX == 0)
          acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(A_[0][q], B_[0][q], acc[0][0], 0, 0, 0);
        else
          accx[q % NX - 1] = __builtin_amdgcn_mfma_f32_32x32x2f32(A_[0][q], B_[0][q], accx[q % NX - 1], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(A_[i][q], B_[j][q], acc[i][j], 0, 0, 0);
    }
  };

  // S register sets in rotation: set s holds chunk c + s; after its MFMAs are issued it is
  // refilled with chunk c + s + S, so S - 1 chunks of loads are always in flight.  The bulk
  // loop body must be branch-free (refills past the end re-load the last full chunk, harmlessly), so
  // that every s_waitcnt waits for exactly the set it consumes: the operand forms (packed A / B) and the
  // A copy-out are therefore compile-time flags of a loop VERSION (run_loop, dispatched once below).  With them
  // as run-time branches inside the loop (rounds 1-4) the compiler could not count the loads across the
  // branch merges and drained every load at the top of each rotation (s_waitcnt vmcnt(0)): one chunk in three
  // waited for all loads in flight (tools/gemm_trace.py per-chunk stamps: 0.32 / 0.32 / 0.52 us).
  const int cfull = min(ce, K / CGL_GEMM_KCHUNK);   // end of this wave's full chunks
  std::integral_constant<bool, false> full;
  std::integral_constant<bool, true> tailc;
  auto run_loop = [&](auto fl) {
    if (cb < cfull) {
      float xa[S][TM][8], xy[S][ABN == 2 ? TM : 1][8], xb[S][TN][8];
#pragma unroll
      for (int s = 0; s < S; ++s) load_chunk(full, min(cb + s, cfull - 1), xa[s], xy[s], xb[s], fl);
      int c = cb;
      for (; c + S <= cfull; c += S) {
#pragma unroll
        for (int s = 0; s < S; ++s) {
          compute_chunk(full, c + s, xa[s], xy[s], xb[s], fl);
#ifdef CGL_GEMM_TRACE
          if (trc && tid == 0 && c == cb && s == 0) trc[3] = wall_clock64();   // chunk 0's operands arrived
#ifdef CGL_GEMM_TRACE_CHUNKS
          if (trc && tid == 0 && c + s - cb < CGL_GEMM_TRACE_W - 8) trc[8 + c + s - cb] = wall_clock64();
#endif
#endif
          // the refill stays right behind the chunk it replaces: without the fences the scheduler sinks all S
          // refills to the end of the rotation, where the next rotation's first chunk waits on them at once
          __builtin_amdgcn_sched_barrier(0);
          load_chunk(full, min(c + s + S, cfull - 1), xa[s], xy[s], xb[s], fl);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
#pragma unroll
      for (int s = 0; s < S - 1; ++s)
        if (c + s < cfull) compute_chunk(full, c + s, xa[s], xy[s], xb[s], fl);
    }
    if (cfull < ce) {   // the K tail (at most one chunk, owned by the last k-group)
      float xa[TM][8], xy[ABN == 2 ? TM : 1][8], xb[TN][8];
      load_chunk(tailc, cfull, xa, xy, xb, fl);
      compute_chunk(tailc, cfull, xa, xy, xb, fl);
    }
  };
  const bool cp = LAYOUT != 2 && a_copy != nullptr;
  if constexpr (LAYOUT == 0) {
    if (apk && bpk)
      cp ? run_loop(CglLoopFl<true, true, true>()) : run_loop(CglLoopFl<true, true, false>());
    else if (apk)
      cp ? run_loop(CglLoopFl<true, false, true>()) : run_loop(CglLoopFl<true, false, false>());
    else if (bpk)
      cp ? run_loop(CglLoopFl<false, true, true>()) : run_loop(CglLoopFl<false, true, false>());
    else
      cp ? run_loop(CglLoopFl<false, false, true>()) : run_loop(CglLoopFl<false, false, false>());
  } else {
    cp ? run_loop(CglLoopFl<false, false, true>()) : run_loop(CglLoopFl<false, false, false>());
  }
  }   // (register-pipelined main loop)

  if constexpr (NX > 1) {
#pragma unroll
    for (int x = 0; x < NX - 1; ++x)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[0][0][r] += accx[x][r];
  }

  // ---------------- split-K reduction (fixed order: wk = 1, 2, 3)
  if (WK > 1) {
    constexpr int NB = TM * TN;
    if (wk > 0) {
      float* dst = s_red + ((wmn * (WK - 1) + (wk - 1)) * NB * 16) * 64;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) dst[((i * TN + j) * 16 + r) * 64 + lane] = acc[i][j][r];
    }
    __syncthreads();
    if (wk == 0) {
      for (int q = 1; q < WK; ++q) {
        const float* src = s_red + ((wmn * (WK - 1) + (q - 1)) * NB * 16) * 64;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] += src[((i * TN + j) * 16 + r) * 64 + lane];
      }
    }
  }

#ifdef CGL_GEMM_TRACE
  if (trc && tid == 0) trc[4] = wall_clock64();
#endif
  // ---------------- cross-workgroup split-K combine (ksplit > 1)
  // Every k-slice workgroup publishes its tile partial with 16-byte write-through (sc1) buffer
  // stores, drains them (vmcnt(0) in every storing wave, then the workgroup barrier) and takes a
  // ticket (relaxed agent-scope atomic); the workgroup drawing ticket KS-1 reads all KS partials
  // back with sc1 loads, sums them in slice order (deterministic: replicas stay bitwise equal)
  // and continues into the epilogue; the others exit.  The ticket is re-zeroed by the reducer.
  // (cdna_hip_programming.md Guideline 16 / "In-launch split-K reduction", sc1 form.)
  if (SK && KS > 1) {
    constexpr int NB = TM * TN;
    typedef int i32x4 __attribute__((ext_vector_type(4)));
    const int wt = WM * WN;
    const long slab = (long)NB * 16 * 64;                      // floats per wave-tile partial
    const long per_slice = (long)ntile * wt * slab;
    auto rs = __builtin_amdgcn_make_buffer_rsrc(d->kpart, (short)0, (int)(per_slice * KS * 4), 0x00020000);
    if (wk == 0) {
      const long off0 = (long)kslice * per_slice + ((long)tile * wt + wmn) * slab;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const f32x4 v = {acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]};
            const int off = (int)((off0 + (((i * TN + j) * 4 + q) * 64 + lane) * 4) * 4);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, v), rs, off, 0, 16);
          }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0)
      s_flag[0] = (__hip_atomic_fetch_add(d->kcount + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                   (unsigned)(KS - 1));
    __syncthreads();
    if (!s_flag[0]) return;
    if (wk == 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
      for (int ksl = 0; ksl < KS; ++ksl) {
        const long off0 = (long)ksl * per_slice + ((long)tile * wt + wmn) * slab;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int off = (int)((off0 + (((i * TN + j) * 4 + q) * 64 + lane) * 4) * 4);
              const f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16));
              acc[i][j][4 * q] += v[0];
              acc[i][j][4 * q + 1] += v[1];
              acc[i][j][4 * q + 2] += v[2];
              acc[i][j][4 * q + 3] += v[3];
            }
      }
    }
    if (tid == 0) __hip_atomic_store(d->kcount + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }

  // ---------------- epilogue (waves with wk == 0 own the tile)
  // register r of block (i, j): row m0 + 32 i + 4 lh + (r & 3) + 8 (r >> 2), column n0 + 32 j + li
  const bool owner = (wk == 0);
  const int rbase = m0 + 4 * lh;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + 32 * j + li;
    const bool colok = col < N;
    const bool ones_col = b_ones && col == N - 1;
    if (owner && colok && !ones_col) {
      float bb;
      if constexpr (EPF) bb = pf_bias[j];
      else bb = h_bias ? gld(h_bias + col) : 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        float* v = (float*)&acc[i][j];
        if (h_bias) {
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] += bb;
        }
        if (e_act == CGL_EPI_ACT_LEAKY) {
          const float sl = e_slope;
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * sl;
        } else if (e_act == CGL_EPI_ACT_TANH) {
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = tanhf(v[r]);   // (double tanh here costs ~4 us on G L4)
        } else if (e_act == CGL_EPI_ACT_SIGMOID) {
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = 1.f / (1.f + expf(-v[r]));
        }
        if (h_mref) {
          const float sl = e_slope;
          float ref[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            if constexpr (EPF) {
              ref[r] = pf_ref[i][j][r];
            } else {
              const int row = min(rbase + 32 * i + (r & 3) + 8 * (r >> 2), M - 1);
              ref[r] = gld(h_mref + (long)row * h_mld + col);
            }
          }
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = ref[r] > 0.f ? v[r] : v[r] * sl;
        }
        if (h_tref) {
          float t[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            if constexpr (EPF) {
              t[r] = pf_ref[i][j][r];
            } else {
              const int row = min(rbase + 32 * i + (r & 3) + 8 * (r >> 2), M - 1);
              t[r] = gld(h_tref + (long)row * h_tld + col);
            }
          }
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = cgl_dtanh(v[r], t[r]);
        }
      }
    }
  }

  // the tile's stores first: they drain while the BatchNorm partials below are reduced (the partials only
  // read the accumulators)
  // (stored row of result row r: ((r & pmask) << pq) + (r >> pl); the identity without a permutation)
  const int pl = e_cperm ? (e_cperm & 255) : 31, pq = e_cperm ? (e_cperm >> 8) : 0;
  const int pmask = e_cperm ? (1 << pl) - 1 : 0x7fffffff;
  if (owner) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + 32 * j + li;
      if (col >= N) continue;
      const bool ones_col = b_ones && col == N - 1;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const float* v = (const float*)&acc[i][j];
        if (ones_col) {
          if (e_bout) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int row = rbase + 32 * i + (r & 3) + 8 * (r >> 2);
              if (row < M) gst(e_bout + (((row & pmask) << pq) + (row >> pl)), v[r]);
            }
            if constexpr (ADAM) cgl_epi_adam(d, d->ad_pb, d->ad_mb, d->ad_vb, rbase + 32 * i, M, 0, 1, v);
          }
        } else {
          float* __restrict__ C = e_C;
          const int ldc = e_ldc;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row0 = rbase + 32 * i + (r & 3) + 8 * (r >> 2);
            const bool rok = row0 < M;
            const int row = ((row0 & pmask) << pq) + (row0 >> pl);
#ifndef CGL_C_STORE_WB
            // write-through (agent-scope) output stores: no dirty C lines are left in the XCD's L2 for the
            // end-of-kernel write-back, and the next launch (on any XCD) reads them from MALL either way.
            // Measured -1.0 us per B = 256 round, interleaved x3 twice (profiles/r04_store_wt_ab.txt); making
            // every plain store write-through (CGL_GST_WT) gave nothing.  -DCGL_C_STORE_WB: plain stores.
            if (rok)
              __hip_atomic_store((CGL_GLOBAL float*)(C + (long)row * ldc + col), v[r], __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
#else
            if (rok) gst(C + (long)row * ldc + col, v[r]);
#endif
          }
          if constexpr (ADAM) cgl_epi_adam(d, d->ad_p, d->ad_m, d->ad_v, rbase + 32 * i, M, col, ldc, v);
        }
      }
    }
  }

  // backward BatchNorm partials of the stored gradient dy (the next GEMM's a_bn 2): per
  // (row tile, column) {sum dy, sum (y - mean) dy} in double over the workgroup's rows (lane
  // rows, then the two lane halves, then the WM waves of the column, fixed order)
  if (e_bnb) {
    const int ldy = d->bnb_ld;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + 32 * j + li;
      const int colc = min(col, N - 1);
      const float mu = gld(d->bnb_mean + colc);
      double Sd = 0.0, Dd = 0.0;
      if (owner && col < N) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          float yv[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = min(rbase + 32 * i + (r & 3) + 8 * (r >> 2), M - 1);
            yv[r] = gld(d->bnb_y + (long)row * ldy + colc);
          }
          const float* v = (const float*)&acc[i][j];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = rbase + 32 * i + (r & 3) + 8 * (r >> 2);
            if (row < M) {
              Sd += (double)v[r];
              Dd += (double)((yv[r] - mu) * v[r]);
            }
          }
        }
      }
      Sd += __shfl_xor(Sd, 32);
      Dd += __shfl_xor(Dd, 32);
      if (WM == 1) {           // one wave row per column tile: its sums are the tile's (no LDS, no barrier)
        if (owner && lh == 0 && col < N) {
          double* p = e_bnb + ((long)tm * N + col) * 2;
          *(CGL_GLOBAL double*)p = Sd;
          *(CGL_GLOBAL double*)(p + 1) = Dd;
        }
      } else if (owner && lh == 0) {
        s_bnd[(((wm * WN + wn) * TN + j) * 32 + li) * 2] = Sd;
        s_bnd[(((wm * WN + wn) * TN + j) * 32 + li) * 2 + 1] = Dd;
      }
    }
    if (WM > 1) __syncthreads();
    if (WM > 1 && owner && wm == 0 && lh == 0) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n0 + 32 * j + li;
        double Sd = 0.0, Dd = 0.0;
        for (int q = 0; q < WM; ++q) {
          Sd += s_bnd[(((q * WN + wn) * TN + j) * 32 + li) * 2];
          Dd += s_bnd[(((q * WN + wn) * TN + j) * 32 + li) * 2 + 1];
        }
        if (col < N) {
          double* p = e_bnb + ((long)tm * N + col) * 2;
          *(CGL_GLOBAL double*)p = Sd;
          *(CGL_GLOBAL double*)(p + 1) = Dd;
        }
      }
    }
  }

  // forward BatchNorm partials of the stored output: per column, per group slot {sum, M2 about the
  // tile-slot mean} over the workgroup's BM rows.  Each lane reduces its own rows two-pass (count, sum,
  // M2 about its own mean), the two lane halves and then the WM waves of the column are merged by
  // Chan's pairwise update in a fixed order: one workgroup barrier per slot, and a slot holding none
  // of the tile's rows (a tile spans <= 2 forward calls; usually one) costs nothing.
  if (e_stat) {
    const int gr = e_gr;
    const int trow0 = tm * BM;
    const int gfirst = trow0 / gr;
    const int gsplit = (gfirst + 1) * gr;   // first row of slot 1
    float* s_st = (float*)s_bnd;            // [WM WN TN 32][3] {n, sum, M2} (s_bnd is free here)
    if (e_bnb && WM > 1) __syncthreads();
    for (int s = 0; s < 2; ++s) {
      const int ra = max(trow0, (gfirst + s) * gr), rb = min(min(trow0 + BM, M), (gfirst + s + 1) * gr);
      if (rb - ra <= 0) {                   // workgroup-uniform
        if (owner && wm == 0 && lh == 0)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int col = n0 + 32 * j + li;
            if (col < N) {
              float* p = e_stat + ((long)(tm * 2 + s) * N + col) * 2;
              gst(p, 0.f);
              gst(p + 1, 0.f);
            }
          }
        continue;
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const bool colok = n0 + 32 * j + li < N;
        float cn = 0.f, sum = 0.f, m2 = 0.f;
        if (owner && colok) {
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            const float* v = (const float*)&acc[i][j];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int row = rbase + 32 * i + (r & 3) + 8 * (r >> 2);
              const bool in = row < M && (row >= gsplit) == (s == 1);
              sum += in ? v[r] : 0.f;
              cn += in ? 1.f : 0.f;
            }
          }
          const float mu = cn > 0.f ? sum / cn : 0.f;
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            const float* v = (const float*)&acc[i][j];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int row = rbase + 32 * i + (r & 3) + 8 * (r >> 2);
              const bool in = row < M && (row >= gsplit) == (s == 1);
              const float dd = v[r] - mu;
              m2 += in ? dd * dd : 0.f;
            }
          }
        }
        {   // lane half 0 (a) with lane half 1 (b)
          const float cb = __shfl_xor(cn, 32), sb = __shfl_xor(sum, 32), mb = __shfl_xor(m2, 32);
          const float ca = lh ? cb : cn, sa = lh ? sb : sum, ma = lh ? mb : m2;
          const float c2 = lh ? cn : cb, s2 = lh ? sum : sb, m22 = lh ? m2 : mb;
          const float nt = ca + c2;
          const float dl = (ca > 0.f && c2 > 0.f) ? s2 / c2 - sa / ca : 0.f;
          cn = nt;
          sum = sa + s2;
          m2 = ma + m22 + (nt > 0.f ? dl * dl * (ca * c2 / nt) : 0.f);
        }
        if (WM == 1) {         // one wave row per column tile: its merge is the tile's (no LDS, no barrier;
          const int col = n0 + 32 * j + li;   // the same values the one-entry merge below would store)
          if (owner && lh == 0 && col < N) {
            float* p = e_stat + ((long)(tm * 2 + s) * N + col) * 2;
            gst(p, 0.f + sum);
            gst(p + 1, 0.f + m2);
          }
        } else if (owner && lh == 0) {
          float* e = s_st + (((wm * WN + wn) * TN + j) * 32 + li) * 3;
          e[0] = cn;
          e[1] = sum;
          e[2] = m2;
        }
      }
      if (WM == 1) continue;
      __syncthreads();
      if (owner && wm == 0 && lh == 0) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = n0 + 32 * j + li;
          float cn = 0.f, sum = 0.f, m2 = 0.f;
          for (int q = 0; q < WM; ++q) {
            const float* e = s_st + (((q * WN + wn) * TN + j) * 32 + li) * 3;
            const float c2 = e[0], s2 = e[1];
            const float nt = cn + c2;
            const float dl = (cn > 0.f && c2 > 0.f) ? s2 / c2 - sum / cn : 0.f;
            m2 += e[2] + (nt > 0.f ? dl * dl * (cn * c2 / nt) : 0.f);
            sum += s2;
            cn = nt;
          }
          if (col < N) {
            float* p = e_stat + ((long)(tm * 2 + s) * N + col) * 2;
            gst(p, sum);
            gst(p + 1, m2);
          }
        }
      }
      __syncthreads();
    }
  }

  // dynamic loss scaling (16-bit operand instantiations only): a non-finite stored weight gradient
  // raises the model's found flag (GradScaler's found_inf), read by that model's Adam launch
  if constexpr (DT != CGL_DTYPE_F32) {
    if (owner && d->inf_flag) {
      bool bad = false;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const bool colok = n0 + 32 * j + li < N;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const float* v = (const float*)&acc[i][j];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = rbase + 32 * i + (r & 3) + 8 * (r >> 2);
            bad |= colok && row < M && !isfinite(v[r]);
          }
        }
      }
      if (bad) atomicOr(d->inf_flag, 1u);
    }
  }
#ifdef CGL_GEMM_TRACE
  if (trc) {
    __syncthreads();
    if (tid == 0) trc[5] = wall_clock64();
  }
#endif
}

// One kernel per per-wave block shape (TM x TN), shared by every GEMM of the step; a grouped
// launch may mix layouts (e.g. the weight gradient (TN) and the input gradient (NN) of one
// layer side by side).  Separate symbols keep the 1x1 variant's register budget (and so its
// occupancy) independent of the 2x2 variant's.
// Dynamic LDS: the operand-transform tables, then the split-K partials of the waves with wk > 0.
// sel (kernel arguments): the launch's problem selection -- first workgroup of problems 1 and 2 (INT_MAX: absent), each
// problem's layout | vec << 2 in 4 bits, and whether d[0] carries a deferred head reduction -- so that a workgroup finds
// its problem and body without reading the descriptor array first.
template <int TM, int TN, bool SK = false, int DT = CGL_DTYPE_F32, int ABN = 0>
__global__ __launch_bounds__(CGL_GEMM_THREADS) void cgl_gemm_f32(const CglGemmDesc* __restrict__ descs, int sel_wg1,
                                                                 int sel_wg2, int sel_meta, int sel_fin,
                                                                 const int* __restrict__ pf, int pf_lines) {
  // (the selection as scalar kernel arguments: with kernarg preloading they arrive in SGPRs at wave start)
  const CglGemmSel sel{sel_wg1, sel_wg2, sel_meta, sel_fin};
#ifdef CGL_GEMM_TRACE
  const unsigned long long t_entry = wall_clock64();
#else
  const unsigned long long t_entry = 0;
#endif
  extern __shared__ float cgl_dyn_lds[];
  __shared__ int s_flag[1];                     // split-K: this workgroup reduces its tile
  __shared__ double s_bnd[4 * TN * 32 * 2];     // per-column BatchNorm partials across waves (WM WN <= 4)
  const int bid = blockIdx.x;
  // the previous head launch's deferred batch-mean loss reduction rides in one extra workgroup (the last)
  if (sel.fin && bid == (int)gridDim.x - 1) {
    cgl_head_finish(descs[0].fin_head, descs[0].fin_head->nwg, cgl_dyn_lds);
    return;
  }
  // L2 warm-up of the next GEMM launch's descriptors: they are read once per round, through the scalar cache,
  // at the head of that launch's dependent chain (descriptor -> operand addresses -> operands); after a round's
  // streaming they have left L2.  Workgroups 0..7 land on XCDs 0..7 (round-robin dispatch), one line per lane;
  // the value is held to the end of the kernel, so the load is issued here and never waited on early.
  int pfv = 0;
  if (bid < 8 && (int)threadIdx.x < pf_lines) pfv = pf[threadIdx.x * 32];
  const int di = bid >= sel.wg2 ? 2 : (bid >= sel.wg1 ? 1 : 0);
  const CglGemmDesc* __restrict__ d = descs + di;
  const int meta = (sel.meta >> (4 * di)) & 15;
  const int layout = meta & 3;
  // VEC: every operand allows 16-byte loads along its contiguous dimension
  const int vec = (meta >> 2) & 1;
#define CGL_BODY(L)                                               \
  do {                                                            \
    if (vec)                                                      \
      cgl_gemm_body<L, 1, TM, TN, SK, DT, ABN>(d, bid, cgl_dyn_lds, s_flag, s_bnd, t_entry);    \
    else                                                          \
      cgl_gemm_body<L, 0, TM, TN, SK, DT, ABN>(d, bid, cgl_dyn_lds, s_flag, s_bnd, t_entry);    \
  } while (0)
  if (layout == 0)
    CGL_BODY(0);
  else if (layout == 1)
    CGL_BODY(1);
  else
    CGL_BODY(2);
#undef CGL_BODY
  asm volatile("" ::"v"(pfv));
}

// One problem whose descriptor travels in the kernel arguments (the single-op entry points cgl_linear_*):
// nothing is uploaded before the launch, so the ops need no host synchronisation and can be captured into
// a graph.  fp32, no split-K, no operand transform, no deferred head.
template <int TM, int TN>
__global__ __launch_bounds__(CGL_GEMM_THREADS) void cgl_gemm_f32_arg(const CglGemmDesc desc) {
  extern __shared__ float cgl_dyn_lds[];
  __shared__ int s_flag[1];
  __shared__ double s_bnd[4 * TN * 32 * 2];
  const CglGemmDesc* __restrict__ d = &desc;
  const int bid = blockIdx.x;
  const int vec = d->a_vec && d->b_vec;
#define CGL_BODY_ARG(L)                                                                             \
  do {                                                                                              \
    if (vec)                                                                                        \
      cgl_gemm_body<L, 1, TM, TN, false, CGL_DTYPE_F32, 0>(d, bid, cgl_dyn_lds, s_flag, s_bnd);     \
    else                                                                                            \
      cgl_gemm_body<L, 0, TM, TN, false, CGL_DTYPE_F32, 0>(d, bid, cgl_dyn_lds, s_flag, s_bnd);     \
  } while (0)
  if (d->layout == 0)
    CGL_BODY_ARG(0);
  else if (d->layout == 1)
    CGL_BODY_ARG(1);
  else
    CGL_BODY_ARG(2);
#undef CGL_BODY_ARG
}

// Host helpers: the LDS tables of a problem's operand transform, its dynamic LDS bytes, its
// workgroups, and the split-K partial floats it needs.
inline int cgl_gemm_tab_floats(const CglGemmDesc& d) {
  if (d.a_bn == 1) return 2 * (CGL_BN_MAXF + 16);
  if (d.a_bn == 2) return 5 * CGL_BNB_TAB;
  return 0;
}
inline int cgl_gemm_stage_bytes(const CglGemmDesc& d) {
  const int sk = (d.WK > 1) ? d.WM * d.WN * (d.WK - 1) * d.TM * d.TN * 16 * 64 * 4 : 0;
  return sk + 4 * cgl_gemm_tab_floats(d);
}
inline int cgl_gemm_wgs(const CglGemmDesc& d) { return d.tiles_m * d.tiles_n * (d.ksplit > 1 ? d.ksplit : 1); }
inline long cgl_gemm_kpart_floats(const CglGemmDesc& d) {
  return d.ksplit > 1 ? (long)d.ksplit * d.tiles_m * d.tiles_n * d.WM * d.WN * d.TM * d.TN * 16 * 64 : 0;
}
