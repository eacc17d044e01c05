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
    if (s.idx0) rr = s.idx0[(s.idx_off ? *s.idx_off : 0) + r];
    return s.p0 + (long)rr * s.ld;
  }
  return s.p1 + (long)(r - s.split) * s.ld;
}

// 8 consecutive k of one row (k-contiguous operand); zeros outside [0,K) or for invalid rows.
__device__ __forceinline__ void cgl_load_kc(const float* __restrict__ rp, bool ok, int k, int K, int vec,
                                            float v[8]) {
  if (vec) {
    float4 x = make_float4(0.f, 0.f, 0.f, 0.f), y = x;
    if (ok && k + 3 < K) x = *reinterpret_cast<const float4*>(rp + k);
    if (ok && k + 7 < K) y = *reinterpret_cast<const float4*>(rp + k + 4);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
    v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (ok && k + j < K) ? rp[k + j] : 0.f;
  }
}

// rows k..k+7 at one column of a row-major [K][ld] operand (mn-contiguous operand).
__device__ __forceinline__ void cgl_load_mn(const float* __restrict__ p, int ld, bool ok, int k, int K,
                                            float v[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (ok && k + j < K) ? p[(long)(k + j) * ld] : 0.f;
}

// Mean / biased variance of BatchNorm group g for feature k from the producer partials
// (exact parallel combination of per-tile {sum, M2}, in double like torch's CPU kernel).
__device__ void cgl_bn_group_stats(const CglBnFwd& bn, int K, int k, int g, double& mean, double& m2,
                                   int& n) {
  const int r0 = g * bn.gr, r1 = min(r0 + bn.gr, bn.mtot);
  n = r1 - r0;
  const int t0 = r0 / bn.part_bm, t1 = (r1 - 1) / bn.part_bm;
  double s = 0.0;
  for (int t = t0; t <= t1; ++t) {
    const int slot = g - (t * bn.part_bm) / bn.gr;
    s += (double)bn.part[((long)(t * 2 + slot) * K + k) * 2 + 0];
  }
  mean = s / n;
  double q = 0.0;
  for (int t = t0; t <= t1; ++t) {
    const int slot = g - (t * bn.part_bm) / bn.gr;
    const int a = max(t * bn.part_bm, r0), b = min((t + 1) * bn.part_bm, r1);
    const int c = b - a;
    const float* pp = bn.part + ((long)(t * 2 + slot) * K + k) * 2;
    const double mt = (double)pp[0] / c;
    const double d = mt - mean;
    q += (double)pp[1] + c * d * d;
  }
  m2 = q;
}

template <int LAYOUT>
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
        const float sc = (float)invstd * bn.gamma[k];
        const float sh = bn.beta[k] - (float)mean * sc;
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
            bn.run_mean[k] = (float)(mom * mean + (1.0 - mom) * (double)bn.run_mean[k]);
            const double unb = m2 / (n - 1);
            bn.run_var[k] = (float)(mom * unb + (1.0 - mom) * (double)bn.run_var[k]);
          }
          if (bn.save_mean) {
            bn.save_mean[(long)g * K + k] = (float)mean;
            bn.save_invstd[(long)g * K + k] = (float)(1.0 / sqrt(m2 / n + bn.eps));
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
  const bool b_ok = bn_ < N;
  const float* __restrict__ a_row = nullptr;
  const float* __restrict__ b_row = nullptr;
  if (LAYOUT != 2) a_row = a_ok ? cgl_row(d->a, am) : d->a.p0;
  if (LAYOUT == 0) b_row = b_ok ? cgl_row(d->b, bn_) : d->b.p0;
  const int a_vec = d->a_vec, b_vec = d->b_vec;
  const int b_ones = (LAYOUT != 0) ? d->b_ones_col : 0;
  const bool b_is_ones = b_ones && (bn_ == N - 1);
  const int gsel = a_tf ? (a_ok ? am / d->bn.gr - g0 : 0) : 0;
  const float slope_tf = d->bn.slope;
  float* __restrict__ a_copy = d->a_copy;
  const bool do_copy = (LAYOUT != 2) && a_copy && tn == 0 && wn == 0 && a_ok && am >= d->a_copy_row0;

  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;

  float av[8], bv[8];
  auto load_chunk = [&](int c, float* A_, float* B_) {
    const int k = c * CGL_GEMM_KCHUNK + 8 * lh;
    if (LAYOUT == 2) {
      cgl_load_mn(d->a.p0 + am, d->a.ld, a_ok, k, K, A_);
    } else {
      cgl_load_kc(a_row, a_ok, k, K, a_vec, A_);
    }
    if (LAYOUT == 0) {
      cgl_load_kc(b_row, b_ok, k, K, b_vec, B_);
    } else {
      if (b_is_ones) {
#pragma unroll
        for (int j = 0; j < 8; ++j) B_[j] = (k + j < K) ? 1.f : 0.f;
      } else {
        cgl_load_mn(d->b.p0 + bn_, d->b.ld, b_ok, k, K, B_);
      }
    }
  };

  if (cb < ce) load_chunk(cb, av, bv);
  for (int c = cb; c < ce; ++c) {
    float an[8], bnx[8];
    if (c + 1 < ce) load_chunk(c + 1, an, bnx);
    const int k = c * CGL_GEMM_KCHUNK + 8 * lh;
    if (a_tf) {
      const float* t = s_tf + (gsel * CGL_TF_MAXK) * 2;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (a_ok && k + j < K) {
          float x = fmaf(av[j], t[(k + j) * 2 + 0], t[(k + j) * 2 + 1]);
          av[j] = x > 0.f ? x : x * slope_tf;
        } else {
          av[j] = 0.f;
        }
      }
    }
    if (do_copy) {
      float* dst = a_copy + (long)am * d->a_copy_ld;
      if (a_vec && k + 7 < K) {
        *reinterpret_cast<float4*>(dst + k) = make_float4(av[0], av[1], av[2], av[3]);
        *reinterpret_cast<float4*>(dst + k + 4) = make_float4(av[4], av[5], av[6], av[7]);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (k + j < K) dst[k + j] = av[j];
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j], bv[j], acc, 0, 0, 0);
    if (c + 1 < ce) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        av[j] = an[j];
        bv[j] = bnx[j];
      }
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
      const float bb = d->bias[col];
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
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rbase + (r & 3) + 8 * (r >> 2);
        if (row < M) {
          const float ref = d->mask_ref[(long)row * d->mask_ld + col];
          v[r] = ref > 0.f ? v[r] : v[r] * sl;
        }
      }
    }
    if (d->tanh_ref) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rbase + (r & 3) + 8 * (r >> 2);
        if (row < M) {
          const float t = d->tanh_ref[(long)row * d->tanh_ld + col];
          v[r] = v[r] * (1.f - t * t);
        }
      }
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
        p[0] = part[s][0];
        p[1] = part[s][1];
      }
    }
  }

  if (owner && colok) {
    if (ones_col) {
      if (d->bias_out) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = rbase + (r & 3) + 8 * (r >> 2);
          if (row < M) d->bias_out[row] = v[r];
        }
      }
    } else {
      float* __restrict__ C = d->C;
      const int ldc = d->ldc;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rbase + (r & 3) + 8 * (r >> 2);
        if (row < M) C[(long)row * ldc + col] = v[r];
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
  if (layout == 0)
    cgl_gemm_body<0>(d, bid, s_tf, s_red, s_col);
  else if (layout == 1)
    cgl_gemm_body<1>(d, bid, s_tf, s_red, s_col);
  else
    cgl_gemm_body<2>(d, bid, s_tf, s_red, s_col);
}
