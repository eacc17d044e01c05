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
//    the workgroup reduces the producer's {sum, M2} partials into a per-feature scale/shift
//    table in LDS and applies BatchNorm1d(train) + LeakyReLU while loading (the reference's
//    BN/LeakyReLU kernels disappear), optionally writing the transformed rows out once;
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

// Mean / biased variance of BatchNorm group g for feature k from the producer partials
// (exact parallel combination of per-tile {sum, M2}, in double like torch's CPU kernel).
__device__ void cgl_bn_group_stats(const CglBnFwd& bn, int K, int k, int g, double& mean, double& m2,
                                   int& n) {
  const int r0 = g * bn.gr, r1 = min(r0 + bn.gr, bn.mtot);
  n = r1 - r0;
  const int t0 = r0 / bn.part_bm, t1 = (r1 - 1) / bn.part_bm;
  // each tile contributes one {sum, M2} pair; blocks of 8 independent loads in flight, then the
  // exact parallel combination M2 = sum M2_t + n_t (mean_t - mean)^2 (fixed order)
  const int nt = t1 - t0 + 1;
  double s = 0.0;
  for (int i0 = 0; i0 < nt; i0 += 8) {
    float ps[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int t = t0 + min(i0 + j, nt - 1);
      const int slot = g - (t * bn.part_bm) / bn.gr;
      ps[j] = gld(bn.part + ((long)(t * 2 + slot) * K + k) * 2);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (i0 + j < nt) s += (double)ps[j];
  }
  mean = s / n;
  double q = 0.0;
  for (int i0 = 0; i0 < nt; i0 += 8) {
    float ps[8], pq[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int t = t0 + min(i0 + j, nt - 1);
      const int slot = g - (t * bn.part_bm) / bn.gr;
      const float* pp = bn.part + ((long)(t * 2 + slot) * K + k) * 2;
      ps[j] = gld(pp);
      pq[j] = gld(pp + 1);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (i0 + j < nt) {
        const int t = t0 + i0 + j;
        const int c = min((t + 1) * bn.part_bm, r1) - max(t * bn.part_bm, r0);
        const double dd = (double)ps[j] / c - mean;
        q += (double)pq[j] + c * dd * dd;
      }
    }
  }
  m2 = q;
}

template <int LAYOUT, int VEC>
__device__ __forceinline__ void cgl_gemm_body(const CglGemmDesc* __restrict__ d, int bid, float* __restrict__ s_tf,
                                              float* __restrict__ s_red, float* __restrict__ s_col) {
  const int M = d->M, N = d->N, K = d->K;
  const int WN = d->WN, WK = d->WK, WM = d->WM;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int li = lane & 31, lh = lane >> 5;
  const int wk = wave % WK, wmn = wave / WK;
  const int wm = wmn / WN, wn = wmn % WN;
  const int local = bid - d->wg_begin;
  const int tm = local / d->tiles_n, tn = local % d->tiles_n;
  const int BM = 32 * WM;
  const int m0 = tm * BM + wm * 32;
  const int n0 = (tn * WN + wn) * 32;

  // ---------------- BatchNorm prologue: scale/shift table for the groups of this row tile
  const int a_tf = (LAYOUT != 2) ? d->a_tf : 0;
  int g0 = 0;
  if (a_tf) {
    const CglBnFwd& bn = d->bn;
    const int rlast = min(tm * BM + BM, M) - 1;
    g0 = (tm * BM) / bn.gr;
    const int g1 = rlast / bn.gr;
    for (int k = tid; k < K; k += CGL_GEMM_THREADS) {
      for (int g = g0; g <= g1; ++g) {
        double mean, m2;
        int n;
        cgl_bn_group_stats(bn, K, k, g, mean, m2, n);
        const double invstd = 1.0 / sqrt(m2 / n + bn.eps);
        const float sc = (float)invstd * gld(bn.gamma + k);
        const float sh = gld(bn.beta + k) - (float)mean * sc;
        s_tf[((g - g0) * CGL_TF_MAXK + k) * 2 + 0] = sc;
        s_tf[((g - g0) * CGL_TF_MAXK + k) * 2 + 1] = sh;
      }
    }
    if (local == 0 && (bn.run_mean || bn.save_mean)) {
      // running statistics: every forward call (group) in order, like the reference's
      // sequential Xd-then-Xg calls (capgan.py:215-220).
      const int ngroups = (bn.mtot + bn.gr - 1) / bn.gr;
      for (int k = tid; k < K; k += CGL_GEMM_THREADS) {
        for (int g = 0; g < ngroups; ++g) {
          double mean, m2;
          int n;
          cgl_bn_group_stats(bn, K, k, g, mean, m2, n);
          if (bn.run_mean) {
            const double mom = bn.momentum;
            gst(bn.run_mean + k, (float)(mom * mean + (1.0 - mom) * (double)gld(bn.run_mean + k)));
            const double unb = m2 / (n - 1);
            gst(bn.run_var + k, (float)(mom * unb + (1.0 - mom) * (double)gld(bn.run_var + k)));
          }
          if (bn.save_mean) {
            gst(bn.save_mean + (long)g * K + k, (float)mean);
            gst(bn.save_invstd + (long)g * K + k, (float)(1.0 / sqrt(m2 / n + bn.eps)));
          }
        }
      }
    }
    __syncthreads();
  }

  // ---------------- main loop
  const int nch = (K + CGL_GEMM_KCHUNK - 1) / CGL_GEMM_KCHUNK;
  const int cb = (wk * nch) / WK, ce = ((wk + 1) * nch) / WK;

  // per-lane operand rows / columns
  const int am = m0 + li;          // A row (kc) or A column (mn)
  const int bn_ = n0 + li;         // B row (NT) or B column (NN/TN)
  const bool a_ok = am < M;
  const int b_ones = (LAYOUT != 0) ? d->b_ones_col : 0;
  const int nmem = N - b_ones;     // columns of B actually in memory
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

  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;

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
      const float* t = s_tf + (gsel * CGL_TF_MAXK) * 2;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int kk = min(k + j, K - 1);
        const float x = fmaf(A_[j], t[kk * 2 + 0], t[kk * 2 + 1]);
        A_[j] = (a_ok && k + j < K) ? (x > 0.f ? x : x * slope_tf) : 0.f;
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

  // two register sets in ping-pong: the loads of chunk c+1 are in flight while chunk c's MFMAs
  // run, and no register copy forces an early wait.  Tail loads are clamped re-loads.
  if (cb < ce) {
    float xa[8], xb[8], ya[8], yb[8];
    load_chunk(cb, xa, xb);
    for (int c = cb; c < ce; c += 2) {
      load_chunk(min(c + 1, ce - 1), ya, yb);
      compute_chunk(c, xa, xb);
      load_chunk(min(c + 2, ce - 1), xa, xb);
      if (c + 1 < ce) compute_chunk(c + 1, ya, yb);
    }
  }

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
    float part[2][2];
    for (int s = 0; s < 2; ++s) {
      // pass 1: sum
      float sum = 0.f;
      if (owner && colok) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = rbase + (r & 3) + 8 * (r >> 2);
          if (row < M && row / gr - gfirst == s) sum += v[r];
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
          if (row < M && row / gr - gfirst == s) {
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
__global__ __launch_bounds__(CGL_GEMM_THREADS) void cgl_gemm_f32(const CglGemmDesc* __restrict__ descs, int ndesc) {
  __shared__ float s_tf[2 * CGL_TF_MAXK * 2];   // BatchNorm scale/shift per (group, k)
  __shared__ float s_red[3 * 16 * 64];          // split-K partial accumulators
  __shared__ float s_col[4 * 32 * 2];           // per-column reductions across waves
  const int bid = blockIdx.x;
  int di = 0;
  for (int q = 1; q < ndesc; ++q)
    if (bid >= descs[q].wg_begin) di = q;
  const CglGemmDesc* __restrict__ d = descs + di;
  const int layout = d->layout;
  // VEC: every k-contiguous operand allows 16-byte loads (K % 4 == 0, aligned rows)
  const int vec = layout == 0 ? (d->a_vec && d->b_vec) : d->a_vec;
  if (layout == 0) {
    if (vec)
      cgl_gemm_body<0, 1>(d, bid, s_tf, s_red, s_col);
    else
      cgl_gemm_body<0, 0>(d, bid, s_tf, s_red, s_col);
  } else if (layout == 1) {
    if (vec)
      cgl_gemm_body<1, 1>(d, bid, s_tf, s_red, s_col);
    else
      cgl_gemm_body<1, 0>(d, bid, s_tf, s_red, s_col);
  } else {
    cgl_gemm_body<2, 0>(d, bid, s_tf, s_red, s_col);
  }
}
