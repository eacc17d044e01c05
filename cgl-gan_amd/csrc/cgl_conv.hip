// Conv GAN path of model/lsgan.py on gfx950: 3x3 convolutions as implicit GEMMs on NHWC
// activations (fp32 MFMA), BatchNorm2d, Dropout2d masks, the adversarial losses, NCHW<->NHWC
// layout changes and a multi-tensor Adam -- every op the reference runs implicitly through
// PyTorch for its conv generator / discriminator:
//
//   nn.Upsample(scale_factor=2) + nn.Conv2d(c, c', 3, 1, 1)       model/lsgan.py:11-12, 15-16
//   nn.Conv2d(64, 1, 3, 1, 1) + nn.Tanh                          model/lsgan.py:19-20
//   nn.Conv2d(c, c', 3, 2, 1) + LeakyReLU(0.2) + Dropout2d(0.25) model/lsgan.py:78
//   nn.BatchNorm2d(c, 0.8)                                       model/lsgan.py:13, 17, 80
//   out.view(B, 128, 8, 8) / out.view(B, -1)                     model/lsgan.py:25, 96 (layout only)
//
// Design (MI355X-first):
//  * Activations are NHWC ("channels_last"): a pixel's channels are contiguous, so an implicit
//    im2col row segment of 8 consecutive k (one tap, 8 channels) is two 16-byte loads.
//  * One MFMA kernel (v_mfma_f32_32x32x2_f32, exact f32) computes every forward and input-gradient
//    convolution from a TAP TABLE: output pixels are enumerated on a (possibly strided) grid,
//    each tap reads the input at (oy*isy + dy[t], ox*isx + dx[t]), and the weights are packed per
//    call into B[n][t*Cin + c] (k-contiguous).  Nearest-neighbour x2 upsampling followed by a 3x3
//    convolution is computed in PHASE form: each of the 4 output parities is a 2x2 convolution of
//    the low-resolution input with combined weights (e.g. W[1]+W[2]), and its input gradient is one
//    4x4-tap convolution of the output gradient at stride 2 -- 16 instead of 36 MACs per
//    (pixel, cin, cout), and neither the upsampled tensor nor its gradient is ever materialised.
//    The stride-2 discriminator convolutions' input gradients are likewise 4 parity problems with
//    1, 2, 2 and 4 taps.  Up to 4 problems share one launch (grouped, XCD-aware tile order).
//  * Weight gradients use the same tap tables: an MFMA GEMM over pixels (the reduction dim)
//    split across workgroups, partial tiles reduced in a fixed order (deterministic, no atomics)
//    and folded back onto the 3x3 OIHW weights.
//  * BatchNorm2d statistics: per-chunk {sum, M2} partials in double, Chan-combined per forward
//    call (group) in a fixed order, torch's formulas (biased variance for the output, unbiased for
//    running_var); backward as torch's batch_norm_backward.  Dropout2d masks come from
//    Philox4x32-10 per (image, channel).
//  * Every launch takes its descriptor by value (kernel arguments): no uploads, no host syncs, so
//    the ops are stream-ordered and capturable in a hipGraph.
//
// Compiled in cgl_conv_tu.hip (shares cgl_internal.h / cgl_common.h: cgl_philox, cgl_lerp, ...).

#define CGL_CONV_MAXP 4
#define CGL_AS4 __attribute__((address_space(4)))

struct CglConvProb {
  int M, N, K, Kp;           // enumerated output pixels, output channels, K = taps * Cin, packed row length
  int OH, OW;                // enumerated output grid per image
  int osy, osx, ooy, oox;    // stored output position (oy * osy + ooy, ox * osx + oox)
  int YH, YW, ldy;           // stored output dims and channel count (pixel stride)
  int isy, isx;              // input step per enumerated output pixel
  int IH, IW, ish;           // virtual input bounds; stored input is read at (iy >> ish, ix >> ish)
  int XH, XW, Cin;           // stored input dims / channels
  int Ty, Tx;                // tap grid, t = ty * Tx + tx
  int dy[4], dx[4];          // tap offsets
  int ym[4], xm[4];          // kernel rows / columns combined into each tap (bitmask of kh / kw)
  int wg_begin, tiles_m, tiles_n, splits;
  const float* X;
  const float* Wp;           // packed weights [N][Kp]
  float* Y;                  // output (fwd), or the output gradient dY (wgrad, read only)
  float* part;               // wgrad partials [splits][N][Kp]
  int st_gr, st_off;         // BatchNorm statistics in the epilogue: rows per forward call (group),
                             // first 32-row chunk of this problem within a group's chunks
};

struct CglConvLaunch {
  CglConvProb p[CGL_CONV_MAXP];
  int np, WM, WN, WK;        // waves per workgroup: WM x WN output blocks x WK k-splits
  const float* bias;         // [N] or null
  int act;                   // CGL_EPI_ACT_*
  float slope;
  const float* drop;         // Dropout2d scale per (image, channel) [img][ldy], or null
  int wbias;                 // weight gradient: im2col column K is the constant 1 (bias gradient)
  double* st_part;           // per-(32-row chunk, channel) BatchNorm2d partials of the stored output:
  int st_cpg;                // 32-row chunks per group (all problems)
  int st_mode;               //   0 {sum, M2} (forward statistics), 1 {sum g, sum g (x - mean)} with
  float st_slope;            //   g = the stored dY (* leaky'(post)) (backward statistics)
  const float* st_x;         // mode 1: the BatchNorm input x, the post-activation (or null) and the
  const float* st_post;      // saved per-call mean [groups][N], all at the stored tensor's positions
  const float* st_mean;
  // forward statistics of a call whose first group (the D step's real call) holds a short batch: only its
  // first *st_nv images are real (DataLoader's short final batch, capgan.py:282,326-331); the padding
  // images' rows are left out of the partials (single-problem launches only; null: every row counts)
  const int* st_nv;
  int ilv;                   // forward: the np problems share X and their tile grid -- tiles interleaved
                             // problem-minor (tile t of every problem back to back on one XCD)
  // forward with the input's BatchNorm2d folded into the operand load (the producer's bn2d finalize wrote
  // scale / shift per (group, channel): in_coef = [2][in_groups][Cin]): x -> fmaf(x, scale, shift), then
  // LeakyReLU when in_act -- cgl_eltwise's arithmetic, so the operand equals the applied activation
  const float* in_coef;
  int in_groups, in_gimg;    // BatchNorm groups (forward calls) and input images per group
  int in_act;
  float in_slope;
  int in_g0;                 // weight gradient (one call's rows): the input's BatchNorm group
  // backward statistics without the post-activation tensor: LeakyReLU'(post) from the sign of the forward's
  // fmaf(x, scale, shift), scale = st_psc[c], shift = st_psc[st_psc_ld + c] (cgl_bn2d_bwd's post_coef)
  const float* st_psc;
  int st_psc_ld;
};

typedef const CGL_AS4 CglConvLaunch* CglKL;
typedef const CGL_AS4 CglConvProb* CglKP;

// The launch descriptor is the kernel's first (by-value) argument: read it through the kernarg
// segment pointer so that uniform-indexed fields become scalar loads (a dynamically indexed
// by-value struct would otherwise be copied to scratch).
__device__ __forceinline__ CglKL cgl_conv_args() { return (CglKL)__builtin_amdgcn_kernarg_segment_ptr(); }

__device__ __forceinline__ int cgl_conv_prob(CglKL L, int bid) {
  int pi = 0;
  for (int q = 1; q < L->np; ++q)
    if (bid >= L->p[q].wg_begin) pi = q;
  return pi;
}

__device__ __forceinline__ void cgl_conv_pix(CglKP P, int m, int& img, int& oy, int& ox) {
  const int hw = P->OH * P->OW;
  img = m / hw;
  const int r = m - img * hw;
  oy = r / P->OW;
  ox = r - oy * P->OW;
}

// q = a / d, r = a % d for 0 <= a < 2^31, d >= 1 (inv = 1.0 / d): the double product is within
// one of the quotient, fixed by one branch-free correction step (no integer division sequence)
__device__ __forceinline__ void cgl_divmod(int a, int d, double inv, int& q, int& r) {
  q = (int)((double)a * inv);
  r = a - q * d;
  const bool hi = r >= d, lo = r < 0;
  q += hi ? 1 : (lo ? -1 : 0);
  r += hi ? -d : (lo ? d : 0);
}

__device__ __forceinline__ int cgl_xcd_tile(int local, int nwg) {
  if (nwg < 16) return local;
  const int xcd = local & 7, pos = local >> 3, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
}

// ------------------------------------------------------------------------------------------
// Forward / input-gradient convolution: C[m][n] = sum_k A[m][k] Wp[n][k] with the implicit A of
// the tap table.  One wave owns TM x TN 32x32 accumulators; WM x WN waves per workgroup.
// FAST: Cin % 16 == 0, so a 16-k chunk lies inside one tap (uniform tap, 2 x 16-byte loads per
// lane and block).  Otherwise each k is decoded per element (tiny-K layers: Cin = 1).
// The folded BatchNorm's activation slope: LeakyReLU(w) = max(w, w * slope) -- bitwise cgl_eltwise's
// (w > 0 ? w : w * slope) for 0 < slope <= 1 (the entry points require it: at slope 0 the select turns
// w = -inf into -inf * 0 = NaN where the max form gives -inf), two VALU ops instead of three;
// act none = slope 1 (max(w, w) = w), so the staging loops carry no activation branch.
__device__ __forceinline__ float cgl_bnin_slope(CglKL L) {
  return L->in_act == CGL_EPI_ACT_LEAKY ? L->in_slope : 1.f;
}

#ifndef CGL_HALO_SB
#define CGL_HALO_SB 8   // the halo window's staging loads in flight per thread (1: one load, then its store)
#endif
template <int TM, int TN, bool FAST, bool BNIN = false, bool HALO = false, bool LDSM = false>
__device__ __forceinline__ void cgl_conv_fwd_body(CglKL L, CglKP P, int local, float* s_red, bool direct = false) {
  constexpr int S = 3;
  static_assert(!LDSM || (TM == 2 && TN == 2 && FAST && !BNIN && !HALO), "the LDS main loop: 2x2 blocks, FAST");
  static_assert(!BNIN || FAST, "the folded BatchNorm input needs the FAST (uniform-tap chunk) path");
  static_assert(!HALO || (TM == 2 && TN == 2 && FAST), "the halo path is the 2x2-block FAST path");
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, li = lane & 31, lh = lane >> 5;
  const int WN = L->WN, WM = L->WM, WK = L->WK;
  // HALO: the workgroup's waves each own the same tile of a different problem (the caller picks P per wave)
  const int wsel = HALO ? 0 : wave;
  const int wk = wsel % WK, wmn = wsel / WK;
  const int wm = wmn / WN, wn = wmn - wm * WN;
  const int tiles_n = P->tiles_n;
  const int tile = direct ? local : cgl_xcd_tile(local, P->tiles_m * tiles_n);
  const int tn = tile % tiles_n, tm = tile / tiles_n;
  const int M = P->M, N = P->N, K = P->K, Kp = P->Kp, Cin = P->Cin;
  const int IH = P->IH, IW = P->IW, ish = P->ish, XW = P->XW, Tx = P->Tx;
  const int m0 = tm * 32 * TM * WM + wm * 32 * TM;
  const int n0 = (tn * WN + wn) * 32 * TN;
  const float* __restrict__ X = P->X;

  int ay[TM], ax[TM];
  long aoff[TM];
  int cgo[TM];                 // BNIN: this row's BatchNorm group offset into the coefficient table
  float* s_coef = s_red;       // BNIN: [2][in_groups][Cin] scale / shift staged in LDS ahead of s_red
  const int coef_n = BNIN ? 2 * L->in_groups * Cin : 0;
  const float bn_sl = BNIN ? cgl_bnin_slope(L) : 0.f;
  if constexpr (BNIN && !HALO) {
    for (int q = tid; q < coef_n; q += 256) s_coef[q] = gld(L->in_coef + q);
    s_red += (coef_n + 63) & ~63;
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    int img, oy, ox;
    cgl_conv_pix(P, min(m0 + 32 * i + li, M - 1), img, oy, ox);
    ay[i] = oy * P->isy;
    ax[i] = ox * P->isx;
    aoff[i] = (long)img * P->XH * XW * Cin;
    cgo[i] = BNIN ? min(img / L->in_gimg, L->in_groups - 1) * Cin : 0;
  }
  const float* brow[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) brow[j] = P->Wp + (long)min(n0 + 32 * j + li, N - 1) * Kp;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto load = [&](int c, float (&A)[TM][8], float (&B)[TN][8], int& okm) {
    const int k0 = c * 16;
    okm = 0;
    if (FAST) {
      // the chunk lies inside one tap (Cin % 16 == 0), or the problem has a single tap and
      // Cin % 4 == 0: then the K tail is masked per float4 (bits 4 / 5 of okm)
      const int t = k0 / Cin;
      const int ci = k0 - t * Cin + 8 * lh;
      const int ty = t / Tx, tx = t - ty * Tx;
      const int dyv = P->dy[ty], dxv = P->dx[tx];
      okm = (ci < Cin ? 16 : 0) | (ci + 4 < Cin ? 32 : 0);
      const int c0 = min(ci, Cin - 4), c1 = min(ci + 4, Cin - 4);
      if (BNIN) okm |= (c0 << 8) | (c1 << 20);   // the channels of the two float4, for the folded BatchNorm
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int iy = ay[i] + dyv, ix = ax[i] + dxv;
        const bool ok = (unsigned)iy < (unsigned)IH && (unsigned)ix < (unsigned)IW;
        okm |= ok ? (1 << i) : 0;
        const int cy = min(max(iy, 0), IH - 1) >> ish, cx = min(max(ix, 0), IW - 1) >> ish;
        gcfp p = (gcfp)(X + aoff[i] + ((long)cy * XW + cx) * Cin);
        const f32x4 u = *(gcf4p)(p + c0), w = *(gcf4p)(p + c1);
        A[i][0] = u[0]; A[i][1] = u[1]; A[i][2] = u[2]; A[i][3] = u[3];
        A[i][4] = w[0]; A[i][5] = w[1]; A[i][6] = w[2]; A[i][7] = w[3];
      }
    } else {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int k = k0 + 8 * lh + q;
          const int kk = min(k, K - 1);
          const int t = kk / Cin, ci = kk - t * Cin;
          const int ty = t / Tx, tx = t - ty * Tx;
          const int iy = ay[i] + P->dy[ty], ix = ax[i] + P->dx[tx];
          const bool ok = k < K && (unsigned)iy < (unsigned)IH && (unsigned)ix < (unsigned)IW;
          okm |= ok ? (1 << (i * 8 + q)) : 0;
          const int cy = min(max(iy, 0), IH - 1) >> ish, cx = min(max(ix, 0), IW - 1) >> ish;
          A[i][q] = ((gcfp)X)[aoff[i] + ((long)cy * XW + cx) * Cin + ci];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      gcfp p = (gcfp)(brow[j] + k0 + 8 * lh);
      const f32x4 u = *(gcf4p)p, w = *(gcf4p)(p + 4);
      B[j][0] = u[0]; B[j][1] = u[1]; B[j][2] = u[2]; B[j][3] = u[3];
      B[j][4] = w[0]; B[j][5] = w[1]; B[j][6] = w[2]; B[j][7] = w[3];
    }
  };
  auto compute = [&](float (&A)[TM][8], float (&B)[TN][8], int okm) {
    if constexpr (BNIN) {
      // BatchNorm2d (+ LeakyReLU) of the loaded input, from the staged scale / shift (before the mask:
      // padded taps and out-of-range channels stay zero, as in the applied activation)
      const int c0 = (okm >> 8) & 0xfff, c1 = (okm >> 20) & 0xfff;
      const int shb = coef_n >> 1;
      const float sl = bn_sl;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const f32x4 s0 = *(const f32x4*)(s_coef + cgo[i] + c0), s1 = *(const f32x4*)(s_coef + cgo[i] + c1);
        const f32x4 h0 = *(const f32x4*)(s_coef + shb + cgo[i] + c0), h1 = *(const f32x4*)(s_coef + shb + cgo[i] + c1);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          float v = fmaf(A[i][q], q < 4 ? s0[q] : s1[q - 4], q < 4 ? h0[q] : h1[q - 4]);
          v = fmaxf(v, v * sl);
          A[i][q] = v;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      if (FAST) {
        const bool ok0 = ((okm >> i) & 1) && (okm & 16), ok1 = ((okm >> i) & 1) && (okm & 32);
#pragma unroll
        for (int q = 0; q < 8; ++q) A[i][q] = (q < 4 ? ok0 : ok1) ? A[i][q] : 0.f;
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) A[i][q] = ((okm >> (i * 8 + q)) & 1) ? A[i][q] : 0.f;
      }
    }
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(A[i][q], B[j][q], acc[i][j], 0, 0, 0);
  };

  // S register sets in rotation (S - 1 chunks of loads in flight); Kp % 16 == 0, no K tail.
  // This wave's k-split: chunks [cb, ce).
  const int nch = Kp >> 4;
  const int cb = (wk * nch) / WK, ce = ((wk + 1) * nch) / WK;
  if constexpr (LDSM) {
    // LDS-staged operand panels (2 x 2 waves of 64 x 64, WK = 1; the input gradients of the upsampling convs):
    // per 16-k chunk the workgroup's 256 threads fetch the A panel [128 rows][16 k] (two 16-byte im2col loads
    // each) and the B panel [128 columns][16 k] (two 16-byte weight loads each) into LDS, where each element is
    // read by the 2 waves sharing its row (column) block instead of loaded by each.  Rows padded to 20 floats:
    // the 16 lanes of a 16-byte read phase cover the 64 banks once.  The next chunk's loads are in flight while
    // this one is multiplied (two register sets, two LDS buffers, one barrier per chunk).  Fragment values and
    // MFMA order are the direct path's (lane half lh holds k 8 lh .. 8 lh + 7 of the chunk), so the results are
    // bitwise equal to it.
    constexpr int RS = 20;
    float* const la = s_red;                  // [2][128][RS]
    float* const lb = s_red + 2 * 128 * RS;   // [2][128][RS]
    const int tid2 = threadIdx.x;
    const int sr = tid2 >> 2, sq = tid2 & 3;  // staging: rows sr and sr + 64, float4 sq of the chunk
    const int mt = tm * 32 * TM * WM, nt = tn * 32 * TN * WN;
    int say[2], sax[2];
    long saoff[2];
    const float* sbrow[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      int img, oy, ox;
      cgl_conv_pix(P, min(mt + sr + 64 * h, M - 1), img, oy, ox);
      say[h] = oy * P->isy;
      sax[h] = ox * P->isx;
      saoff[h] = (long)img * P->XH * XW * Cin;
      sbrow[h] = P->Wp + (long)min(nt + sr + 64 * h, N - 1) * Kp;
    }
    auto gload = [&](int c, f32x4 (&ra)[2], f32x4 (&rb)[2], int& okm) {
      const int k0 = c * 16, t = k0 / Cin, ci = k0 - t * Cin + 4 * sq;
      const int ty = t / Tx, tx = t - ty * Tx;
      const int dyv = P->dy[ty], dxv = P->dx[tx];
      okm = 0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int iy = say[h] + dyv, ix = sax[h] + dxv;
        const bool ok = (unsigned)iy < (unsigned)IH && (unsigned)ix < (unsigned)IW;
        okm |= ok ? (1 << h) : 0;
        const int cy = min(max(iy, 0), IH - 1) >> ish, cx = min(max(ix, 0), IW - 1) >> ish;
        ra[h] = *(gcf4p)(X + saoff[h] + ((long)cy * XW + cx) * Cin + ci);
        rb[h] = *(gcf4p)(sbrow[h] + k0 + 4 * sq);
      }
    };
    auto stage = [&](int buf, const f32x4 (&ra)[2], const f32x4 (&rb)[2], int okm) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        *(f32x4*)&la[(buf * 128 + sr + 64 * h) * RS + 4 * sq] = ((okm >> h) & 1) ? ra[h] : f32x4{0.f, 0.f, 0.f, 0.f};
        *(f32x4*)&lb[(buf * 128 + sr + 64 * h) * RS + 4 * sq] = rb[h];
      }
    };
    const int ra0 = wm * 32 * TM + li, rb0 = wn * 32 * TN + li;
    auto mmc = [&](int buf) {
      float A[TM][8], B[TN][8];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const float* w = &la[(buf * 128 + ra0 + 32 * i) * RS + 8 * lh];
        const f32x4 u = *(const f32x4*)w, v = *(const f32x4*)(w + 4);
        A[i][0] = u[0]; A[i][1] = u[1]; A[i][2] = u[2]; A[i][3] = u[3];
        A[i][4] = v[0]; A[i][5] = v[1]; A[i][6] = v[2]; A[i][7] = v[3];
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const float* w = &lb[(buf * 128 + rb0 + 32 * j) * RS + 8 * lh];
        const f32x4 u = *(const f32x4*)w, v = *(const f32x4*)(w + 4);
        B[j][0] = u[0]; B[j][1] = u[1]; B[j][2] = u[2]; B[j][3] = u[3];
        B[j][4] = v[0]; B[j][5] = v[1]; B[j][6] = v[2]; B[j][7] = v[3];
      }
      __builtin_amdgcn_sched_barrier(0);   // all 8 LDS reads ahead of the 32 MFMAs
#pragma unroll
      for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(A[i][q], B[j][q], acc[i][j], 0, 0, 0);
    };
    f32x4 r0a[2], r0b[2], r1a[2], r1b[2];
    int ok0, ok1;
    gload(0, r0a, r0b, ok0);
    gload(min(1, nch - 1), r1a, r1b, ok1);
    stage(0, r0a, r0b, ok0);
    __syncthreads();
    int c = 0;
    for (; c + 2 <= nch; c += 2) {
      gload(min(c + 2, nch - 1), r0a, r0b, ok0);
      mmc(0);
      stage(1, r1a, r1b, ok1);
      __syncthreads();
      gload(min(c + 3, nch - 1), r1a, r1b, ok1);
      mmc(1);
      stage(0, r0a, r0b, ok0);
      __syncthreads();
    }
    if (c < nch) mmc(0);
  } else if constexpr (HALO) {
    // LDS-staged input window (the phase-form upsampling conv: 4 output parities x 2x2 taps, all reading one
    // low-res window).  The workgroup's tile is 64 enumerated rows = R = 64 / OW whole low-res rows of one
    // image; its window (rows y0 - 1 .. y0 + R, columns -1 .. OW, every channel, zeros outside the image) is
    // loaded once -- with the folded BatchNorm applied here, once per element -- and the 4 waves (one per
    // parity) read their A fragments of every tap from it.  The chunk order and MFMA sequence are the
    // direct path's, so the results are bitwise equal.
    const int OWp = P->OW, hwp = P->OH * OWp;
    const int img = m0 / hwp, y0 = (m0 - img * hwp) / OWp;
    const int WC = OWp + 2, WR = 64 / OWp + 2, CS = Cin + 4;   // pixel stride padded (LDS banks)
    const int c4 = Cin >> 2;
    const float* __restrict__ Xi = X + (long)img * P->XH * XW * Cin;
    const int g = BNIN ? min(img / L->in_gimg, L->in_groups - 1) : 0;
    // BNIN: when the staging stride keeps each thread on one channel quad, its scale / shift are loaded once
    const bool qfix = (256 % c4) == 0;
    // the activation flag and slope in registers: read through the kernarg pointer inside the loop, the slope's
    // scalar load sat under the LeakyReLU condition and became a branch per value
    const float in_sl = BNIN ? cgl_bnin_slope(L) : 0.f;
    f32x4 sc0 = {0.f, 0.f, 0.f, 0.f}, sh0 = sc0;
    if (BNIN && qfix) {
      sc0 = *(gcf4p)(L->in_coef + g * Cin + 4 * (tid % c4));
      sh0 = *(gcf4p)(L->in_coef + (L->in_groups + g) * Cin + 4 * (tid % c4));
    }
    // SB staging loads in flight per thread (a load-then-store loop kept ~2 in flight: ~7 serial round trips for
    // a 57 KB window), then the transform and the LDS stores
    constexpr int SB = CGL_HALO_SB;
    const int tot = WR * WC * c4;
    for (int e0 = tid; e0 < tot; e0 += 256 * SB) {
      f32x4 v[SB];
      int okm = 0;
#pragma unroll
      for (int u = 0; u < SB; ++u) {
        const int e = e0 + 256 * u;
        const int q = e % c4, pix = e / c4;
        const int wr = pix / WC, wc = pix - wr * WC;
        const int iy = y0 - 1 + wr, ix = wc - 1;
        v[u] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (e < tot && (unsigned)iy < (unsigned)IH && (unsigned)ix < (unsigned)IW) {
          v[u] = *(gcf4p)(Xi + ((long)iy * XW + ix) * Cin + 4 * q);
          okm |= 1 << u;
        }
      }
#pragma unroll
      for (int u = 0; u < SB; ++u) {
        const int e = e0 + 256 * u;
        if (e >= tot) break;
        const int q = e % c4, pix = e / c4;
        if constexpr (BNIN) {
          if ((okm >> u) & 1) {
            const f32x4 sc = qfix ? sc0 : *(gcf4p)(L->in_coef + g * Cin + 4 * q);
            const f32x4 sh = qfix ? sh0 : *(gcf4p)(L->in_coef + (L->in_groups + g) * Cin + 4 * q);
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              float w = fmaf(v[u][t], sc[t], sh[t]);
              w = fmaxf(w, w * in_sl);
              v[u][t] = w;
            }
          }
        }
        *(f32x4*)(s_red + pix * CS + 4 * q) = v[u];
      }
    }
    __syncthreads();
    // this lane's window pixel (tap offset 0) per row block
    int wpix[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int rr = 32 * i + li;                   // row within the tile
      wpix[i] = (rr / OWp + 1) * WC + (rr % OWp) + 1;
    }
    auto lda = [&](int c, float (&A)[TM][8]) {
      const int k0 = c * 16, t = k0 / Cin, ci = k0 - t * Cin + 8 * lh;
      const int ty = t / Tx, tx = t - ty * Tx;
      const int toff = P->dy[ty] * WC + P->dx[tx];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const float* w = s_red + (wpix[i] + toff) * CS + ci;
        const f32x4 u = *(const f32x4*)w, v = *(const f32x4*)(w + 4);
        A[i][0] = u[0]; A[i][1] = u[1]; A[i][2] = u[2]; A[i][3] = u[3];
        A[i][4] = v[0]; A[i][5] = v[1]; A[i][6] = v[2]; A[i][7] = v[3];
      }
    };
    auto ldb = [&](int c, float (&B)[TN][8]) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        gcfp p = (gcfp)(brow[j] + c * 16 + 8 * lh);
        const f32x4 u = *(gcf4p)p, w = *(gcf4p)(p + 4);
        B[j][0] = u[0]; B[j][1] = u[1]; B[j][2] = u[2]; B[j][3] = u[3];
        B[j][4] = w[0]; B[j][5] = w[1]; B[j][6] = w[2]; B[j][7] = w[3];
      }
    };
    auto mm = [&](float (&A)[TM][8], float (&B)[TN][8]) {
#pragma unroll
      for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(A[i][q], B[j][q], acc[i][j], 0, 0, 0);
    };
    // B (weights, global) S - 1 chunks ahead in a rotation of S register sets, A (LDS) one chunk ahead
    float xb[S][TN][8], xa[2][TM][8];
#pragma unroll
    for (int s2 = 0; s2 < S; ++s2) ldb(min(s2, nch - 1), xb[s2]);
    lda(0, xa[0]);
    int c = 0;
    for (; c + S <= nch; c += S) {
#pragma unroll
      for (int s2 = 0; s2 < S; ++s2) {
        lda(min(c + s2 + 1, nch - 1), xa[(s2 + 1) & 1]);
        mm(xa[s2 & 1], xb[s2]);
        ldb(min(c + s2 + S, nch - 1), xb[s2]);
      }
      if (S & 1) {   // keep the A double buffer's parity aligned with s2 = 0 at the next iteration
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int q = 0; q < 8; ++q) xa[0][i][q] = xa[1][i][q];
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < S - 1; ++s2)
      if (c + s2 < nch) {
        lda(min(c + s2 + 1, nch - 1), xa[(s2 + 1) & 1]);
        mm(xa[s2 & 1], xb[s2]);
      }
  } else if (cb < ce) {
    float xa[S][TM][8], xb[S][TN][8];
    int okm[S];
#pragma unroll
    for (int s = 0; s < S; ++s) load(min(cb + s, ce - 1), xa[s], xb[s], okm[s]);
    int c = cb;
    for (; c + S <= ce; c += S) {
#pragma unroll
      for (int s = 0; s < S; ++s) {
        compute(xa[s], xb[s], okm[s]);
        load(min(c + s + S, ce - 1), xa[s], xb[s], okm[s]);
      }
    }
#pragma unroll
    for (int s = 0; s < S - 1; ++s)
      if (c + s < ce) compute(xa[s], xb[s], okm[s]);
  }
  // k-split reduction through LDS in a fixed order (wk = 1, 2, 3 added to wk = 0): deterministic
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
    if (wk > 0) return;
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

  // epilogue: bias, activation, Dropout2d scale, NHWC store at the mapped position.  The activation
  // is a uniform branch around the element loops; the output pixel of each row is decoded once per
  // 32-row block and stepped from row to row (no per-element divisions); the Dropout2d multipliers of
  // a block are all loaded before its stores (a load after a store may alias it, which would
  // serialise one global round trip per element).
  const int ldy = P->ldy, YH = P->YH, YW = P->YW, OW = P->OW, hw = P->OH * P->OW;
  const double inv_hw = 1.0 / hw, inv_ow = 1.0 / OW;
  const int osy = P->osy, osx = P->osx, ooy = P->ooy, oox = P->oox;
  const float* __restrict__ bias = L->bias;
  const float* __restrict__ drop = L->drop;
  const int act = L->act;
  const float sl = L->slope;
  float* __restrict__ Y = P->Y;
  float bj[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = min(n0 + 32 * j + li, N - 1);
    bj[j] = bias ? gld(bias + col) : 0.f;
  }
#define CGL_EPI_LOOP(EXPR)                                  \
  _Pragma("unroll") for (int i = 0; i < TM; ++i)            \
  _Pragma("unroll") for (int j = 0; j < TN; ++j)            \
  _Pragma("unroll") for (int r = 0; r < 16; ++r) {          \
    float v = acc[i][j][r] + bj[j];                         \
    EXPR;                                                   \
    acc[i][j][r] = v;                                       \
  }
  if (act == CGL_EPI_ACT_LEAKY) { CGL_EPI_LOOP(v = v > 0.f ? v : v * sl) }
  else if (act == CGL_EPI_ACT_TANH) { CGL_EPI_LOOP(v = cgl_tanh(v)) }
  else if (act == CGL_EPI_ACT_SIGMOID) { CGL_EPI_LOOP(v = 1.f / (1.f + expf(-v))) }
  else { CGL_EPI_LOOP((void)0) }
#undef CGL_EPI_LOOP
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int rowb = m0 + 32 * i;               // wave-uniform first row of the block
    if (rowb >= M) break;
    const int row0 = rowb + 4 * lh;
    int pix[16];
    auto decode = [&](int r, int& img) {
      const int row = row0 + (r & 3) + 8 * (r >> 2);
      int rem, oy, ox;
      cgl_divmod(row, hw, inv_hw, img, rem);
      cgl_divmod(rem, OW, inv_ow, oy, ox);
      pix[r] = (img * YH + oy * osy + ooy) * YW + ox * osx + oox;
      return row;
    };
    if (drop) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        int img;
        const int row = decode(r, img);
        const long dro = (long)(row < M ? img : 0) * ldy;
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j][r] *= gld(drop + dro + min(n0 + 32 * j + li, N - 1));
      }
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        int img;
        decode(r, img);
      }
    }
    // BatchNorm2d statistics of the stored values (the next op's BatchNorm, cgl_bn2d_fwd_stats): per
    // 32-row chunk and channel {sum, M2 about the chunk mean} in double, the two lane halves
    // combined by one xor-32 exchange (fixed order); the chunks of a forward call are contiguous
    int imb, remb, oyb, oxb;
    cgl_divmod(rowb, hw, inv_hw, imb, remb);
    cgl_divmod(remb, OW, inv_ow, oyb, oxb);
    const int pixb = __builtin_amdgcn_readfirstlane((imb * YH + oyb * osy + ooy) * YW + oxb * osx + oox);
    if (L->st_part && L->st_mode == 1) {
      // backward statistics (cgl_bn2d_bwd_stats): x and post loaded at the stored positions through
      // buffer resources of the same base (every row of a statistics launch is valid)
      const int g = rowb / P->st_gr;
      const long chunk = (long)g * L->st_cpg + P->st_off + (rowb - g * P->st_gr) / 32;
      const auto rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(L->st_x) + (long)pixb * ldy, (short)0,
                                                        0x7fffffff, 0x00020000);
      const float* pp = L->st_post ? L->st_post : L->st_x;
      const auto rp = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(pp) + (long)pixb * ldy, (short)0,
                                                        0x7fffffff, 0x00020000);
      const float psl = L->st_slope;
      const bool psc = L->st_psc != nullptr;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n0 + 32 * j + li;
        const int colc = min(col, N - 1);
        const float mu = gld(L->st_mean + (long)g * N + colc);
        const float sc = psc ? gld(L->st_psc + colc) : 0.f, sh = psc ? gld(L->st_psc + L->st_psc_ld + colc) : 0.f;
        float xv[16], pv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int off = ((pix[r] - pixb) * ldy + colc) * 4;
          xv[r] = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(rx, off, 0, 0));
          if (!psc) pv[r] = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(rp, off, 0, 0));
        }
        if (psc) {
#pragma unroll
          for (int r = 0; r < 16; ++r) pv[r] = fmaf(xv[r], sc, sh);
        }
        const bool pon = psc || L->st_post;
        double S = 0.0, D = 0.0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float y = acc[i][j][r];
          const float gg = pon ? (pv[r] > 0.f ? y : y * psl) : y;
          S += (double)gg;
          D += (double)(gg * (xv[r] - mu));
        }
        S += __shfl_xor(S, 32);
        D += __shfl_xor(D, 32);
        if (lh == 0 && col < N) {
          double* dst = L->st_part + (chunk * N + col) * 2;
          dst[0] = S;
          dst[1] = D;
        }
      }
    } else if (L->st_part && L->st_nv && rowb < P->st_gr && rowb + 32 > min(gldi(L->st_nv), P->st_gr / hw) * hw) {
      // a chunk of the short first call that holds padding rows: {sum, M2 about the mean} over its real rows
      // only (the finalize derives every chunk's count from the same *st_nv)
      const int nvr = min(gldi(L->st_nv), P->st_gr / hw) * hw;
      const long chunk = P->st_off + rowb / 32;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        double sm = 0.0, cn = 0.0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const bool in = row0 + (r & 3) + 8 * (r >> 2) < nvr;
          sm += in ? (double)acc[i][j][r] : 0.0;
          cn += in ? 1.0 : 0.0;
        }
        sm += __shfl_xor(sm, 32);
        cn += __shfl_xor(cn, 32);
        const double mu = cn > 0.0 ? sm / cn : 0.0;
        double m2 = 0.0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const double dd = (double)acc[i][j][r] - mu;
          m2 += row0 + (r & 3) + 8 * (r >> 2) < nvr ? dd * dd : 0.0;
        }
        m2 += __shfl_xor(m2, 32);
        const int col = n0 + 32 * j + li;
        if (lh == 0 && col < N) {
          double* dst = L->st_part + (chunk * N + col) * 2;
          dst[0] = sm;
          dst[1] = m2;
        }
      }
    } else if (L->st_part) {
      const int g = rowb / P->st_gr;
      const long chunk = (long)g * L->st_cpg + P->st_off + (rowb - g * P->st_gr) / 32;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        double sm = 0.0;
#pragma unroll
        for (int r = 0; r < 16; ++r) sm += (double)acc[i][j][r];
        sm += __shfl_xor(sm, 32);
        const double mu = sm * (1.0 / 32.0);
        double m2 = 0.0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const double dd = (double)acc[i][j][r] - mu;
          m2 += dd * dd;
        }
        m2 += __shfl_xor(m2, 32);
        const int col = n0 + 32 * j + li;
        if (lh == 0 && col < N) {
          double* dst = L->st_part + (chunk * N + col) * 2;
          dst[0] = sm;
          dst[1] = m2;
        }
      }
    }
    // stores through a buffer resource based at the block's first output pixel (output pixels grow
    // with the row, so every offset is >= 0): rows past M / columns past N get an out-of-range
    // offset and are dropped by the hardware -- no per-element branches
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(Y + (long)pixb * ldy, (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const bool rok = row0 + (r & 3) + 8 * (r >> 2) < M;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n0 + 32 * j + li;
        const int off = (rok && col < N) ? ((pix[r] - pixb) * ldy + col) * 4 : (int)0x80000000;
        // (through a scalar copy: a bit_cast of the vector element itself was lowered to element 0)
        const float v = acc[i][j][r];
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(v), rs, off, 0, 0);
      }
    }
  }
}

template <int TM, int TN, bool FAST, bool BNIN = false, bool LDSM = false>
__global__ __launch_bounds__(256) void cgl_conv_fwd(CglConvLaunch args) {
  (void)args;
  extern __shared__ float cgl_conv_lds[];
  CglKL L = cgl_conv_args();
  const int bid = blockIdx.x;
  if (L->ilv) {
    // problems sharing one input (the 4 output parities of an upsampling conv in phase form, the
    // input-parity problems of a stride-2 input gradient): unit u = (tile u / np of problem u % np),
    // units XCD-contiguous, so the np tiles reading one input window run back to back in one L2
    const int np = L->np;
    const int unit = cgl_xcd_tile(bid, L->p[0].tiles_m * L->p[0].tiles_n * np);
    cgl_conv_fwd_body<TM, TN, FAST, BNIN, false, LDSM>(L, &L->p[unit % np], unit / np, cgl_conv_lds, true);
    return;
  }
  const int pi = cgl_conv_prob(L, bid);
  CglKP P = &L->p[pi];
  cgl_conv_fwd_body<TM, TN, FAST, BNIN, false, LDSM>(L, P, bid - P->wg_begin, cgl_conv_lds);
}

// The phase-form upsampling conv with its input window staged in LDS (HALO path of cgl_conv_fwd_body): one
// workgroup per (64-row tile, 64-output-channel slice), its 4 waves = the 4 output-parity problems
// (launch_conv_mma: conv_halo_ok).
template <bool BNIN>
__global__ __launch_bounds__(256) void cgl_conv_fwd_halo(CglConvLaunch args) {
  (void)args;
  extern __shared__ float cgl_conv_lds[];
  CglKL L = cgl_conv_args();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // XCD-contiguous tile order: the N-halves of one row tile and vertically adjacent tiles (which share
  // window rows) run on one XCD's L2
  CglKP P = &L->p[wave];
  cgl_conv_fwd_body<2, 2, true, BNIN, true>(L, P, cgl_xcd_tile(blockIdx.x, P->tiles_m * P->tiles_n), cgl_conv_lds,
                                             true);
}

// ------------------------------------------------------------------------------------------
// Weight gradient: part[s][n][k] = sum over the pixels m of split s of dY[pos(m)][n] * A[m][k]
// (A = the tap table's implicit im2col of X).  Rows of the result tile are output channels
// (operand A = dY, 32 consecutive channels of one pixel per lane group: coalesced), columns are
// im2col columns (operand B, consecutive channels of one tap: coalesced); each lane half takes 8
// consecutive pixels of a 16-pixel chunk (the MFMA k permutation of cgl_gemm.hip).
// Work unit = one wave: (tile, split) with a (32 TM) x (32 TN) result tile; a workgroup runs 4
// consecutive units (no LDS, no barriers), so small layers (Conv2d(1, 16): 16 x 9 results) do not
// pay for a large workgroup tile.
// Read-only zeros: operand loads of padded taps / pixels past M point here instead of being masked
// after the load (saves the mask bookkeeping and the per-MFMA-operand selects of the k-loop).  The
// loads index it with an output channel (< N) or an input channel (< Cin), so it covers
// CGL_ZERO_PAGE floats; conv_bwd_weight_impl refuses larger layers (dense layers reach N = 8192).
#define CGL_ZERO_PAGE 65536
__device__ float cgl_zero_page[CGL_ZERO_PAGE];

// ROW: every problem of the launch has OW % 8 == 0 and M % 16 == 0, so the 8 pixels of a lane
// half are always valid and lie in one output row: one pixel decode per chunk, constant address
// strides along the row, the tap's row bounds checked once (a fraction of the generic path's VALU).
// BNIN: X is the PRE-BatchNorm map (groups of L->in_gimg images, scale / shift in L->in_coef): each valid
// im2col value is fmaf(x, scale, shift) (+ LeakyReLU), cgl_eltwise's arithmetic; padded taps stay zero
template <int TM, int TN, bool ROW, bool BNIN = false>
__device__ __forceinline__ void cgl_conv_wgrad_body(CglKL L, CglKP P, int local) {
#ifndef CGL_WGRAD_S
#define CGL_WGRAD_S 2
#endif
  constexpr int S = CGL_WGRAD_S;   // operand register sets in rotation (S - 1 chunks of loads in flight)
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, li = lane & 31, lh = lane >> 5;
  const int tiles = P->tiles_m * P->tiles_n;
  const int unit = local * 4 + wave;
  if (unit >= tiles * P->splits) return;
  const int split = unit / tiles;
  const int tile = unit - split * tiles;
  const int tn = tile % P->tiles_n, tm = tile / P->tiles_n;
  const int M = P->M, N = P->N, K = P->K, Kp = P->Kp, Cin = P->Cin;
  const int IH = P->IH, IW = P->IW, ish = P->ish, XW = P->XW, XH = P->XH, Tx = P->Tx;
  const int n0 = tm * 32 * TM;
  const int k0c = tn * 32 * TN;
  const float* __restrict__ X = P->X;
  const float* __restrict__ dY = P->Y;
  const int ldy = P->ldy, YH = P->YH, YW = P->YW;
  const int osy = P->osy, osx = P->osx, ooy = P->ooy, oox = P->oox, isy = P->isy, isx = P->isx;
  const int OH = P->OH, OW = P->OW;

  int rch[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) rch[i] = min(n0 + 32 * i + li, N - 1);
  int cdy[TN], cdx[TN], cci[TN];
  bool cok[TN], cone[TN];
  const int wbias = L->wbias;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int kc = k0c + 32 * j + li;
    cok[j] = kc < K;
    cone[j] = wbias && kc == K;   // the bias column: B = 1 for every valid pixel
    const int kk = min(kc, K - 1);
    const int t = kk / Cin;
    cci[j] = kk - t * Cin;
    const int ty = t / Tx, tx = t - ty * Tx;
    cdy[j] = P->dy[ty];
    cdx[j] = P->dx[tx];
  }
  // BNIN: this lane's columns' scale / shift for up to two BatchNorm groups (the D step's two calls: group
  // in_g0 + img / in_gimg)
  float bsc[2][TN], bsh[2][TN];
  const int bg = BNIN ? max(1, min(L->in_groups - L->in_g0, 2)) : 1;
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const long gq = L->in_g0 + min(q, bg - 1);
      bsc[q][j] = BNIN ? gld(L->in_coef + gq * Cin + cci[j]) : 0.f;
      bsh[q][j] = BNIN ? gld(L->in_coef + (L->in_groups + gq) * Cin + cci[j]) : 0.f;
    }
  const float in_sl = BNIN ? cgl_bnin_slope(L) : 0.f;       // (in registers: see the halo staging)
  auto bn = [&](float x, int img, int j) {
    const int q = (bg > 1 && img >= L->in_gimg) ? 1 : 0;     // (<= 2 groups: no division per value)
    float v = fmaf(x, q ? bsc[1][j] : bsc[0][j], q ? bsh[1][j] : bsh[0][j]);
    v = fmaxf(v, v * in_sl);
    return v;
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // operands of invalid pixels / out-of-bounds taps are loaded from cgl_zero_page (no masks)
  const float* __restrict__ zp = cgl_zero_page;
  auto load = [&](int c, float (&A)[TM][8], float (&B)[TN][8], int& okm) {
    okm = 0;
    if (ROW) {
      int img, oy, ox;
      cgl_conv_pix(P, c * 16 + 8 * lh, img, oy, ox);
      const float* ya0 = dY + (((long)img * YH + oy * osy + ooy) * YW + ox * osx + oox) * ldy;
      const long ystep = (long)osx * ldy;
#pragma unroll
      for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int i = 0; i < TM; ++i) A[i][q] = ((gcfp)(ya0 + q * ystep))[rch[i]];
      const float* ximg = X + (long)img * XH * XW * Cin;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int iy = oy * isy + cdy[j];
        const bool rowok = cok[j] && (unsigned)iy < (unsigned)IH;
        const float* rb = ximg + (long)(rowok ? (iy >> ish) : 0) * XW * Cin + cci[j];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int ix = (ox + q) * isx + cdx[j];
          const bool ok = rowok && (unsigned)ix < (unsigned)IW;
          const float* bb = ok ? rb + (long)(ix >> ish) * Cin : zp + cci[j];
          B[j][q] = *(gcfp)bb;
          if (BNIN) B[j][q] = ok ? bn(B[j][q], img, j) : 0.f;
        }
      }
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 8; ++q) B[j][q] = cone[j] ? 1.f : B[j][q];
      return;
    }
    // decode the first pixel of this lane half once, then step along the row (wrapping)
    int img, oy, ox;
    cgl_conv_pix(P, min(c * 16 + 8 * lh, M - 1), img, oy, ox);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int m = c * 16 + 8 * lh + q;
      const bool mv = m < M;
      if (q > 0) {
        // branch-free stepping (the nested ifs compiled to divergent exec-mask branches per pixel: the lane
        // halves step different pixels)
        ++ox;
        const bool wx = ox == OW;
        ox = wx ? 0 : ox;
        oy += wx ? 1 : 0;
        const bool wy = oy == OH;
        oy = wy ? 0 : oy;
        img += wy ? 1 : 0;
        img = mv ? img : 0;
        oy = mv ? oy : 0;
        ox = mv ? ox : 0;
      }
      const long ya = (((long)img * YH + oy * osy + ooy) * YW + ox * osx + oox) * ldy;
      const float* ab = mv ? dY + ya : zp;
#pragma unroll
      for (int i = 0; i < TM; ++i) A[i][q] = ((gcfp)ab)[rch[i]];
      const long xo = (long)img * XH * XW * Cin;
      const int iyb = oy * isy, ixb = ox * isx;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int iy = iyb + cdy[j], ix = ixb + cdx[j];
        const bool ok = mv && cok[j] && (unsigned)iy < (unsigned)IH && (unsigned)ix < (unsigned)IW;
        const float* bb = ok ? X + xo + ((long)(iy >> ish) * XW + (ix >> ish)) * Cin : zp;
        B[j][q] = ((gcfp)bb)[cci[j]];
        if (BNIN) B[j][q] = ok ? bn(B[j][q], img, j) : 0.f;
        B[j][q] = cone[j] ? (mv ? 1.f : 0.f) : B[j][q];
      }
    }
  };
  auto compute = [&](float (&A)[TM][8], float (&B)[TN][8], int okm) {
    (void)okm;
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(A[i][q], B[j][q], acc[i][j], 0, 0, 0);
  };

  const int nchk = (M + 15) >> 4;
  const int splits = P->splits;
  const int cb = (int)(((long)split * nchk) / splits), ce = (int)(((long)(split + 1) * nchk) / splits);
  if (cb < ce) {
    float xa[S][TM][8], xb[S][TN][8];
    int okm[S];
#pragma unroll
    for (int s = 0; s < S; ++s) load(min(cb + s, ce - 1), xa[s], xb[s], okm[s]);
    int c = cb;
    for (; c + S <= ce; c += S) {
#pragma unroll
      for (int s = 0; s < S; ++s) {
        compute(xa[s], xb[s], okm[s]);
        load(min(c + s + S, ce - 1), xa[s], xb[s], okm[s]);
      }
    }
#pragma unroll
    for (int s = 0; s < S - 1; ++s)
      if (c + s < ce) compute(xa[s], xb[s], okm[s]);
  }

  float* __restrict__ part = P->part + (long)split * N * Kp;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int kc = k0c + 32 * j + li;
    if (kc >= K + wbias) continue;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = n0 + 32 * i + 4 * lh + (r & 3) + 8 * (r >> 2);
        if (n < N) gst(part + (long)n * Kp + kc, acc[i][j][r]);
      }
  }
}

template <int TM, int TN, bool ROW = false, bool BNIN = false>
__global__ __launch_bounds__(256) void cgl_conv_wgrad(CglConvLaunch args) {
  (void)args;
  CglKL L = cgl_conv_args();
  const int bid = blockIdx.x;
  const int pi = cgl_conv_prob(L, bid);
  CglKP P = &L->p[pi];
  cgl_conv_wgrad_body<TM, TN, ROW, BNIN>(L, P, bid - P->wg_begin);
}

// ------------------------------------------------------------------------------------------
// Weight gradient with LDS-staged panels (the large upsampling convs of the LSGAN generator: 16K - 64K
// pixels per phase problem, N = 64 / 128 output channels, K = 512).  A workgroup owns an R x C result tile
// (R = 64 WM output channels, C = 64 WN im2col columns; 4 waves of 2 x 2 32x32 blocks) over one pixel
// split.  Per 16-pixel chunk its 256 threads fetch the dY panel [16][R] and the im2col panel [16][C] with
// 16-byte loads (4 channels of one pixel) and stage them in LDS, where WN waves share each dY element and
// WM waves each X element: the wave-unit kernel's 4-byte fragment loads (one per MFMA operand and wave)
// become a quarter of the load instructions and 1 / WN + 1 / WM of the bytes.  Chunk c + 2's loads are in
// flight while chunk c is multiplied (two register sets, two LDS buffers, one barrier per chunk).  Same
// partials [split][N][Kp] and k permutation as cgl_conv_wgrad (pixel 8 lh + q of a chunk is lane half lh's
// k of MFMA step q), so cgl_conv_wgrad_reduce is shared.  Requirements: wgrad_lds_wm.
// KS = 2: 512-thread workgroups of two 4-wave halves that take alternate chunks of one (twice as long) pixel
// split, each half with its own LDS buffers, summed through LDS at the end (half 0 + half 1, fixed order):
// the same waves per SIMD with half the splits, so half the partials to write and to reduce.
#define CGL_WLDS_PAD 4
// BNIN: X is the PRE-BatchNorm map of one forward call (group L->in_g0): the staged im2col values are
// LeakyReLU(fmaf(x, scale, shift)) -- cgl_eltwise's arithmetic, so the panel equals the applied activation
template <int WM, int WN, int KS, bool BNIN = false>
__global__ __launch_bounds__(256 * KS, 2 / KS) void cgl_conv_wgrad_lds(CglConvLaunch args) {
  (void)args;
  static_assert(KS == 1 || KS == 2, "one or two halves");
  constexpr int R = 64 * WM, C = 64 * WN;
  constexpr int RP = R + CGL_WLDS_PAD, CP = C + CGL_WLDS_PAD;   // padded rows: the lane halves (8 rows
                                                                 // apart) land on disjoint banks
  constexpr int FA = R / 4, FB = C / 4;                          // float4 per pixel row of each panel
  constexpr int NA = 16 * FA / 256, NB = 16 * FB / 256;          // float4 loads per thread and chunk
  static_assert(WM * WN == 4 && NA >= 1 && NB >= 1, "4 waves, whole panels");
  constexpr int HALF = 2 * 16 * (RP + CP);                       // one half's two A and two B buffers
  static_assert(KS == 1 || KS * HALF >= 256 * 64, "the halves' merge reuses the staging LDS");
  __shared__ __attribute__((aligned(16))) float pool[KS * HALF];
  CglKL L = cgl_conv_args();
  const int pi = cgl_conv_prob(L, blockIdx.x);
  CglKP P = &L->p[pi];
  const int tiles = P->tiles_m * P->tiles_n;
  const int local = cgl_xcd_tile(blockIdx.x - P->wg_begin, tiles * P->splits);
  const int split = local / tiles, tile = local - split * tiles;
  const int n0 = (tile / P->tiles_n) * R, k0 = (tile % P->tiles_n) * C;
  const int half = KS == 1 ? 0 : __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 8);
  const int tid = threadIdx.x & 255;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, li = lane & 31, lhf = lane >> 5;
  const int wm = wave / WN, wn = wave - (wave / WN) * WN;
  float* const sa0 = pool + half * HALF;                          // [2][16 RP]
  float* const sb0 = sa0 + 2 * 16 * RP;                           // [2][16 CP]
  const int N = P->N, Kp = P->Kp, Cin = P->Cin;
  const int IH = P->IH, IW = P->IW, ish = P->ish, XW = P->XW, XH = P->XH;
  const int ldy = P->ldy, YH = P->YH, YW = P->YW;
  const int osy = P->osy, osx = P->osx, ooy = P->ooy, oox = P->oox, isy = P->isy, isx = P->isx;
  const int lw = __builtin_ctz(P->OW), lhw = __builtin_ctz(P->OW) + __builtin_ctz(P->OH);
  const int mw = P->OW - 1, mh = P->OH - 1;
  const float* __restrict__ X = P->X;
  const float* __restrict__ dY = P->Y;
  // this thread's fixed panel columns: dY channel n0 + 4 fa, im2col columns k0 + 4 fb .. + 3 (one tap)
  const int fa = tid % FA, pa = tid / FA;
  const int fb = tid % FB, pb = tid / FB;
  const int kk = k0 + 4 * fb;
  const int tap = kk / Cin, ci = kk - tap * Cin;
  const int cdy = P->dy[tap / P->Tx], cdx = P->dx[tap - (tap / P->Tx) * P->Tx];
  f32x4 bsc = {0.f, 0.f, 0.f, 0.f}, bsh = bsc;
  const float in_sl = BNIN ? cgl_bnin_slope(L) : 0.f;       // (in registers: see the halo staging)
  if constexpr (BNIN) {
    bsc = *(gcf4p)(L->in_coef + (long)L->in_g0 * Cin + ci);
    bsh = *(gcf4p)(L->in_coef + (long)(L->in_groups + L->in_g0) * Cin + ci);
  }
  // A 16-pixel chunk never crosses an image (OH OW >= 16, powers of two): pixel c 16 + p decodes as the chunk's
  // (img0, oy0, ox0) -- uniform, scalar -- plus (p >> lw, p & mw) without carries, so each load slot keeps a
  // constant element offset from the chunk's base pointer and only the X bounds test is per chunk and lane.
  int aoff[NA], bky[NB], bkx[NB], boff[NB];
#pragma unroll
  for (int r = 0; r < NA; ++r) {
    const int p = pa + (256 / FA) * r, py = p >> lw, px = p & mw;
    aoff[r] = (py * osy * YW + px * osx) * ldy + n0 + 4 * fa;
  }
#pragma unroll
  for (int r = 0; r < NB; ++r) {
    const int p = pb + (256 / FB) * r, py = p >> lw, px = p & mw;
    bky[r] = py * isy + cdy;
    bkx[r] = px * isx + cdx;
    boff[r] = (bky[r] * XW + bkx[r]) * Cin + ci;
  }
  (void)ish; (void)XH;

  // (the out-of-bounds taps' zeros are applied when staging, so nothing waits on a load before the MFMAs)
  auto load = [&](int c, f32x4 (&ra)[NA], f32x4 (&rb)[NB], int& okb) {
    const int m0 = c * 16;
    const int img0 = m0 >> lhw, oy0 = (m0 >> lw) & mh, ox0 = m0 & mw;
    const float* ya = dY + ((long)(img0 * YH + oy0 * osy + ooy) * YW + ox0 * osx + oox) * ldy;
#pragma unroll
    for (int r = 0; r < NA; ++r) ra[r] = *(gcf4p)(ya + aoff[r]);
    const int Y0 = oy0 * isy, X0 = ox0 * isx;
    const float* xa = X + ((long)img0 * XH * XW + (long)Y0 * XW + X0) * Cin;
    okb = 0;
#pragma unroll
    for (int r = 0; r < NB; ++r) {
      const bool ok = (unsigned)(Y0 + bky[r]) < (unsigned)IH && (unsigned)(X0 + bkx[r]) < (unsigned)IW;
      okb |= ok ? (1 << r) : 0;
      rb[r] = *(gcf4p)(ok ? xa + boff[r] : X + ci);
    }
  };
  auto stage = [&](int buf, const f32x4 (&ra)[NA], const f32x4 (&rb)[NB], int okb) {
#pragma unroll
    for (int r = 0; r < NA; ++r) *(f32x4*)&sa0[buf * 16 * RP + (pa + (256 / FA) * r) * RP + 4 * fa] = ra[r];
#pragma unroll
    for (int r = 0; r < NB; ++r) {
      f32x4 v = rb[r];
      if constexpr (BNIN) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          float w = fmaf(v[u], bsc[u], bsh[u]);
          w = fmaxf(w, w * in_sl);
          v[u] = w;
        }
      }
      *(f32x4*)&sb0[buf * 16 * CP + (pb + (256 / FB) * r) * CP + 4 * fb] =
          ((okb >> r) & 1) ? v : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  // all 32 operands of the chunk are read from LDS before the first MFMA (the reads of step q + 1 do not
  // wait behind step q's MFMAs; the waits are progressive)
  auto compute = [&](int buf) {
    const float* A = &sa0[buf * 16 * RP + 8 * lhf * RP + wm * 64 + li];
    const float* B = &sb0[buf * 16 * CP + 8 * lhf * CP + wn * 64 + li];
    float a[8][2], b[8][2];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      a[q][0] = A[q * RP];
      a[q][1] = A[q * RP + 32];
      b[q][0] = B[q * CP];
      b[q][1] = B[q * CP + 32];
    }
    __builtin_amdgcn_sched_barrier(0);   // keep the reads ahead (the scheduler would sink them to their MFMAs)
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q][0], b[q][0], acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q][0], b[q][1], acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q][1], b[q][0], acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q][1], b[q][1], acc[1][1], 0, 0, 0);
    }
  };

  const int nchk = P->M >> 4, splits = P->splits;
  const int cb = (int)(((long)split * nchk) / splits), ce = (int)(((long)(split + 1) * nchk) / splits);
  // this half's chunks: cb + half + KS i, i < ni (the same count for both halves: every barrier is shared;
  // a half whose last chunk lies past ce loads a clamped one and skips its MFMAs)
  const int ni = (ce - cb + KS - 1) / KS;
  auto chunk = [&](int i) { return min(cb + half + KS * i, ce - 1); };
  auto live = [&](int i) { return cb + half + KS * i < ce; };
  if (ni > 0) {
    f32x4 r0a[NA], r0b[NB], r1a[NA], r1b[NB];
    int ok0, ok1;
    load(chunk(0), r0a, r0b, ok0);
    load(chunk(min(1, ni - 1)), r1a, r1b, ok1);
    stage(0, r0a, r0b, ok0);
    __syncthreads();
    int i = 0;
    for (; i + 2 <= ni; i += 2) {
      // buffer 0 holds step i, r1 step i + 1
      load(chunk(min(i + 2, ni - 1)), r0a, r0b, ok0);
      if (KS == 1 || live(i)) compute(0);   // (KS 1: no branch, so the staging interleaves with the MFMAs)
      stage(1, r1a, r1b, ok1);
      __syncthreads();
      load(chunk(min(i + 3, ni - 1)), r1a, r1b, ok1);
      if (KS == 1 || live(i + 1)) compute(1);
      stage(0, r0a, r0b, ok0);
      __syncthreads();
    }
    if (i < ni && (KS == 1 || live(i))) compute(0);   // an odd last step
  }
  if constexpr (KS == 2) {
    // half 1 hands its accumulators to half 0 through the (now idle) staging LDS
    __syncthreads();
    if (half == 1) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) pool[((i * 2 + j) * 16 + r) * 256 + tid] = acc[i][j][r];
    }
    __syncthreads();
    if (half == 1) return;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] += pool[((i * 2 + j) * 16 + r) * 256 + tid];
  }
  float* __restrict__ part = P->part + (long)split * N * Kp;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int kc = k0 + wn * 64 + 32 * j + li;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = n0 + wm * 64 + 32 * i + 4 * lhf + (r & 3) + 8 * (r >> 2);
        gst(part + (long)n * Kp + kc, acc[i][j][r]);
      }
  }
}

// ------------------------------------------------------------------------------------------
// One-output-channel convolution on the vector ALUs (N == 1: Conv2d(64, 1) of the generator's
// last layer, and the input gradient of the discriminator's Conv2d(1, 16)) -- an MFMA tile would
// waste 31 of its 32 columns.  Channels run across lanes: L = Cin / 4 lanes own one pixel (one
// float4 of channels each, so a wave's load covers 64 / L whole pixel vectors, fully coalesced),
// the lane's slice of every tap's weights stays in registers, and the L partial sums are combined
// by an xor tree (fixed order).  Requires Cin % 4 == 0, Cin / 4 a power of two <= 64, <= 16 taps.
// iterations per wave: each iteration's loads wait on the previous one's, so the D Conv2d(1, 16) input
// gradient (512 workgroups at 8) ran latency-serialised; 2 gives 4x the workgroups
#define CGL_N1_IT 2
__global__ __launch_bounds__(256) void cgl_conv_n1(CglConvLaunch args) {
  (void)args;
  CglKL L = cgl_conv_args();
  const int bid = blockIdx.x;
  const int pi = cgl_conv_prob(L, bid);
  CglKP P = &L->p[pi];
  const int Cin = P->Cin, Tx = P->Tx, T = P->Ty * P->Tx;
  const int c4 = Cin >> 2;
  const int lanes = c4 < 64 ? c4 : 64;         // lanes per pixel (power of two)
  const int nb = c4 / lanes;                   // float4 blocks per lane and tap (T * nb <= 16)
  const int TB = T * nb;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = lane & (lanes - 1), slot = lane / lanes, ppw = 64 / lanes;
  const int IH = P->IH, IW = P->IW, ish = P->ish, XW = P->XW;
  f32x4 w[16];
#pragma unroll
  for (int tb = 0; tb < 16; ++tb) {
    const int t = tb / nb, b = tb - t * nb;
    w[tb] = tb < TB ? *(gcf4p)(P->Wp + t * Cin + 4 * (q + b * lanes)) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const float bias = L->bias ? gld(L->bias) : 0.f;
  const int M = P->M;
  const int per_wg = 4 * ppw * CGL_N1_IT;      // CGL_N1_IT iterations of every wave per workgroup
  const int m_begin = (bid - P->wg_begin) * per_wg;
  for (int it = 0; it < CGL_N1_IT; ++it) {
    const int m = m_begin + (it * 4 + wave) * ppw + slot;
    const bool mv = m < M;
    int img, oy, ox;
    cgl_conv_pix(P, min(m, M - 1), img, oy, ox);
    const float* __restrict__ X = P->X + (long)img * P->XH * XW * Cin + 4 * q;
    f32x4 v[16];
#pragma unroll
    for (int tb = 0; tb < 16; ++tb) {
      if (tb < TB) {
        const int t = tb / nb, b = tb - t * nb;
        const int ty = t / Tx, tx = t - ty * Tx;
        const int iy = oy * P->isy + P->dy[ty], ix = ox * P->isx + P->dx[tx];
        const bool ok = (unsigned)iy < (unsigned)IH && (unsigned)ix < (unsigned)IW;
        const int cy = min(max(iy, 0), IH - 1) >> ish, cx = min(max(ix, 0), IW - 1) >> ish;
        v[tb] = *(gcf4p)(X + ((long)cy * XW + cx) * Cin + 4 * b * lanes);
        if (!ok) v[tb] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    float acc = 0.f;
#pragma unroll
    for (int tb = 0; tb < 16; ++tb) {
      if (tb < TB) {
        acc = fmaf(v[tb][0], w[tb][0], acc);
        acc = fmaf(v[tb][1], w[tb][1], acc);
        acc = fmaf(v[tb][2], w[tb][2], acc);
        acc = fmaf(v[tb][3], w[tb][3], acc);
      }
    }
    for (int o = 1; o < lanes; o <<= 1) acc += __shfl_xor(acc, o);
    if (mv && q == 0) {
      float y = acc + bias;
      if (L->act == CGL_EPI_ACT_LEAKY) y = y > 0.f ? y : y * L->slope;
      else if (L->act == CGL_EPI_ACT_TANH) y = cgl_tanh(y);
      else if (L->act == CGL_EPI_ACT_SIGMOID) y = 1.f / (1.f + expf(-y));
      if (L->drop) y *= gld(L->drop + (long)img * P->ldy);
      gst(P->Y + (((long)img * P->YH + oy * P->osy + P->ooy) * P->YW + ox * P->osx + P->oox) * P->ldy, y);
    }
  }
}

// LDS-tiled variant for a stride-1 3x3 one-output-channel convolution (Conv2d(64, 1, 3, 1, 1) +
// Tanh, model/lsgan.py:19-20): a workgroup stages the (TH + 2) x (W + 2) input halo of TH output
// rows of one image in LDS (coalesced 16-byte loads, zero padding written explicitly), so every
// input pixel is read from memory once per tile instead of once per tap; then L = Cin / 4 lanes per
// output pixel read their channel slice of the 9 taps from LDS and combine by an xor tree.
// C4T / WT: compile-time channel-quads / width (0: read from the descriptor) -- the G's Conv2d(64, 1)
// at 32x32 runs the specialised instance, whose index arithmetic is shifts and constant divisions.
#define CGL_N1T_TH 4
template <int C4T, int WT>
__global__ __launch_bounds__(256) void cgl_conv_n1_tile(CglConvLaunch args) {
  (void)args;
  extern __shared__ float cgl_conv_lds[];
  CglKL L = cgl_conv_args();
  CglKP P = &L->p[0];
  const int W = WT ? WT : P->OW, H = P->OH;
  const int c4 = C4T ? C4T : (P->Cin >> 2), lanes = c4;   // c4 <= 64, power of two
  const int Cin = 4 * c4;
  const int tiles_y = (H + CGL_N1T_TH - 1) / CGL_N1T_TH;
  const int img = blockIdx.x / tiles_y, y0 = (blockIdx.x - img * tiles_y) * CGL_N1T_TH;
  const int HR = CGL_N1T_TH + 2, WR = W + 2;
  const float* __restrict__ X = P->X + (long)img * P->XH * P->XW * Cin;
  // stage rows y0-1 .. y0+TH, cols -1 .. W (zero outside the image): every load of the thread is
  // issued first from a clamped (valid) address and zero-selected afterwards -- a load under a
  // branch drains vmcnt per element and serialises the staging (tot4 <= 16 * 256 by the launch
  // condition: LDS <= 64 KB)
  const int tot4 = HR * WR * c4;
  f32x4 v[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int e = min((int)threadIdx.x + 256 * k, tot4 - 1);
    const int q = e & (c4 - 1), pix = e / c4;
    const int ry = pix / WR, rx = pix - ry * WR;
    const int iy = y0 - 1 + ry, ix = rx - 1;
    const bool ok = (unsigned)iy < (unsigned)P->XH && (unsigned)ix < (unsigned)P->XW;
    const int cy = min(max(iy, 0), P->XH - 1), cx = min(max(ix, 0), P->XW - 1);
    v[k] = *(gcf4p)(X + ((long)cy * P->XW + cx) * Cin + 4 * q);
    if (!ok) v[k] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int e = (int)threadIdx.x + 256 * k;
    if (e < tot4) *(f32x4*)&cgl_conv_lds[(long)(e / c4) * Cin + 4 * (e & (c4 - 1))] = v[k];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int q = lane & (lanes - 1);
  const int slot = threadIdx.x / lanes, nslot = 256 / lanes;
  f32x4 w[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) w[t] = *(gcf4p)(P->Wp + t * Cin + 4 * q);
  const float bias = L->bias ? gld(L->bias) : 0.f;
  const int npix = CGL_N1T_TH * W;
  const int iters = (npix + nslot - 1) / nslot;   // uniform across the workgroup (xor tree below)
  for (int it = 0; it < iters; ++it) {
    const int pp = it * nslot + slot;
    const bool valid = pp < npix;
    const int p = valid ? pp : npix - 1;
    const int ty = p / W, tx = p - ty * W;
    float acc = 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ky = t / 3, kx = t - 3 * ky;
      const f32x4 v = *(const f32x4*)&cgl_conv_lds[((long)(ty + ky) * WR + tx + kx) * Cin + 4 * q];
      acc = fmaf(v[0], w[t][0], acc);
      acc = fmaf(v[1], w[t][1], acc);
      acc = fmaf(v[2], w[t][2], acc);
      acc = fmaf(v[3], w[t][3], acc);
    }
    for (int o = 1; o < lanes; o <<= 1) acc += __shfl_xor(acc, o);
    if (valid && q == 0 && y0 + ty < H) {
      float yv = acc + bias;
      if (L->act == CGL_EPI_ACT_LEAKY) yv = yv > 0.f ? yv : yv * L->slope;
      else if (L->act == CGL_EPI_ACT_TANH) yv = cgl_tanh(yv);
      else if (L->act == CGL_EPI_ACT_SIGMOID) yv = 1.f / (1.f + expf(-yv));
      if (L->drop) yv *= gld(L->drop + (long)img * P->ldy);
      gst(P->Y + (((long)img * P->YH + y0 + ty) * P->YW + tx) * P->ldy, yv);
    }
  }
}

// Tap-partial form of the stride-1 3x3 Conv2d(64, 1) + Tanh at 32x32 (model/lsgan.py:19-20): the
// input is read once per tile as a stream and each pixel is contracted with all 9 taps at once,
// s_t(i) = sum_c X(i, c) W[0][c][t], leaving 9 floats per pixel in LDS; an output pixel is then
// y(o) = sum_t s_t(o + d_t) (zero outside the image).  4 lanes own one input pixel (16 channels =
// four 16-byte loads each; a wave's loads cover 16 whole pixels), so the channel reduction is two
// xor steps; every load of a lane is issued before its first FMA.  A workgroup covers TH = 8 output
// rows of one image: (TH + 2) / TH = 1.25 reads per input pixel, 12 KB of LDS.
#define CGL_N1P_TH 8
__global__ __launch_bounds__(256) void cgl_conv_n1_part(CglConvLaunch args) {
  (void)args;
  constexpr int W = 32, C = 64, TH = CGL_N1P_TH, HR = TH + 2, WR = W + 2, NP = HR * W / 64;
  __shared__ float part[9][HR * WR];
  CglKL L = cgl_conv_args();
  CglKP P = &L->p[0];
  const int H = P->OH;
  const int tiles_y = (H + TH - 1) / TH;
  const int img = blockIdx.x / tiles_y, y0 = (blockIdx.x - img * tiles_y) * TH;
  const float* __restrict__ X = P->X + (long)img * H * W * C;
  const int j = threadIdx.x & 3, g = threadIdx.x >> 2;       // lane in the pixel group, group 0..63
  f32x4 x[NP][4];
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    const int pix = k * 64 + g, ry = pix / W, rx = pix - ry * W;
    const int iy = min(max(y0 - 1 + ry, 0), H - 1);
#pragma unroll
    for (int i = 0; i < 4; ++i) x[k][i] = *(gcf4p)(X + ((long)iy * W + rx) * C + 16 * j + 4 * i);
  }
  if (threadIdx.x < 2 * HR) {                                 // zero padding columns -1 and W
    const int r = threadIdx.x >> 1, col = (threadIdx.x & 1) ? WR - 1 : 0;
#pragma unroll
    for (int t = 0; t < 9; ++t) part[t][r * WR + col] = 0.f;
  }
  if (L->in_coef) {   // the input's BatchNorm2d (+ LeakyReLU) folded into the load (one group per image)
    const int cg = min(img / L->in_gimg, L->in_groups - 1) * C, shb = L->in_groups * C;
    const float sl = cgl_bnin_slope(L);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f32x4 sc = *(gcf4p)(L->in_coef + cg + 16 * j + 4 * i), sh = *(gcf4p)(L->in_coef + shb + cg + 16 * j + 4 * i);
#pragma unroll
      for (int k = 0; k < NP; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = fmaf(x[k][i][e], sc[e], sh[e]);
          v = fmaxf(v, v * sl);
          x[k][i][e] = v;
        }
    }
  }
  f32x4 w[9][4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) w[t][i] = *(gcf4p)(P->Wp + t * C + 16 * j + 4 * i);
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    const int pix = k * 64 + g, ry = pix / W, rx = pix - ry * W;
    const bool ok = (unsigned)(y0 - 1 + ry) < (unsigned)H;
    float sv[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      // pairwise over the lane's 16 channels (4 independent 4-term chains), then the 4-lane tree
      float a4[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a4[i] = x[k][i][0] * w[t][i][0];
        a4[i] = fmaf(x[k][i][1], w[t][i][1], a4[i]);
        a4[i] = fmaf(x[k][i][2], w[t][i][2], a4[i]);
        a4[i] = fmaf(x[k][i][3], w[t][i][3], a4[i]);
      }
      float a = (a4[0] + a4[1]) + (a4[2] + a4[3]);
      a += __shfl_xor(a, 1);
      a += __shfl_xor(a, 2);
      sv[t] = ok ? a : 0.f;
    }
#pragma unroll
    for (int t = 0; t < 9; ++t)
      if ((t & 3) == j) part[t][ry * WR + rx + 1] = sv[t];
  }
  __syncthreads();
  const int ty = threadIdx.x / W, tx = threadIdx.x - ty * W;  // one output pixel per thread
  float st[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) st[t] = part[t][(ty + t / 3) * WR + tx + t % 3];
  const float acc = (((st[0] + st[1]) + (st[2] + st[3])) + ((st[4] + st[5]) + (st[6] + st[7]))) + st[8];
  if (y0 + ty < H) {
    float yv = acc + (L->bias ? gld(L->bias) : 0.f);
    if (L->act == CGL_EPI_ACT_LEAKY) yv = yv > 0.f ? yv : yv * L->slope;
    else if (L->act == CGL_EPI_ACT_TANH) yv = cgl_tanh(yv);
    else if (L->act == CGL_EPI_ACT_SIGMOID) yv = 1.f / (1.f + expf(-yv));
    if (L->drop) yv *= gld(L->drop + (long)img * P->ldy);
    gst(P->Y + (((long)img * P->YH + y0 + ty) * P->YW + tx) * P->ldy, yv);
  }
}

// Weight gradient of a one-output-channel convolution (Conv2d(64, 1): 576 results reduced over every
// output pixel) on the vector ALUs: thread = one im2col column k, pixels of the split in order, 8
// loads in flight; partials part[split][0][k] for the fixed-order reduction.
__global__ __launch_bounds__(256) void cgl_conv_wgrad_n1(CglConvLaunch args) {
  (void)args;
  CglKL L = cgl_conv_args();
  CglKP P = &L->p[0];
  const int K = P->K, Cin = P->Cin, Tx = P->Tx;
  const int k = blockIdx.x * 256 + threadIdx.x;
  const int split = blockIdx.y, splits = P->splits;
  const int M = P->M;
  const int mb = (int)(((long)split * M) / splits), me = (int)(((long)(split + 1) * M) / splits);
  const int kk = min(k, K - 1);
  const int t = kk / Cin, c = kk - t * Cin;
  const int ty = t / Tx, tx = t - ty * Tx;
  const int dyv = P->dy[ty], dxv = P->dx[tx];
  const int IH = P->IH, IW = P->IW, ish = P->ish, XW = P->XW, XH = P->XH;
  float acc = 0.f;
  for (int m0 = mb; m0 < me; m0 += 8) {
    float d[8], x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = min(m0 + i, me - 1);
      int img, oy, ox;
      cgl_conv_pix(P, m, img, oy, ox);
      d[i] = gld(P->Y + (((long)img * P->YH + oy * P->osy + P->ooy) * P->YW + ox * P->osx + P->oox) * P->ldy);
      const int iy = oy * P->isy + dyv, ix = ox * P->isx + dxv;
      const bool ok = (unsigned)iy < (unsigned)IH && (unsigned)ix < (unsigned)IW;
      const int cy = min(max(iy, 0), IH - 1) >> ish, cx = min(max(ix, 0), IW - 1) >> ish;
      x[i] = gld(P->X + (((long)img * XH + cy) * XW + cx) * Cin + c);
      if (!ok || m0 + i >= me) x[i] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) acc = fmaf(d[i], x[i], acc);
  }
  if (k < K) gst(P->part + (long)split * P->Kp + k, acc);
}

// Input-stationary weight gradient of a stride-1 one-output-channel convolution (Conv2d(64, 1, 3, 1, 1)):
// L = Cin / 4 lanes own one INPUT pixel (a float4 of channels each, loaded once, coalesced); every
// tap t pairs it with the output-gradient pixel q - off_t (a broadcast scalar).  9 x 4 accumulators
// per lane; the 256 / L pixel slots of a block are combined through LDS in a fixed order, giving
// part[block][t * Cin + c] for the fixed-order split reduction.
// C4T / XWT / XHT: compile-time channel quads and input width / height (0: from the descriptor).
// The specialised instance (3x3 taps, host-checked) sizes its LDS reduction to 256 / L slots x 9 taps x
// Cin = 36 KB (four workgroups per CU instead of two with the generic 64 KB) and keeps 4 input pixels
// per slot in flight -- the kernel is a stream of X, so bytes in flight per CU set its rate.
// STG > 0: the output-gradient window of the block's pixel range (linear dY indices qb - OW - 1 ..
// qe + OW, host-checked to fit STG floats, dY dense with the input's height / width) is staged in LDS
// once, so the T per-pixel gathers are LDS broadcasts instead of vector-memory instructions.
// BNIN: X is the PRE-BatchNorm map of one forward call (group L->in_g0), applied per loaded float4 (each
// lane's channel quad is fixed, so its scale / shift are loaded once)
template <int C4T, int XWT, int XHT, int CGL_N1T_PX, int REDN, int STG, bool BNIN = false>
__global__ __launch_bounds__(256) void cgl_conv_wgrad_n1t(CglConvLaunch args) {
  (void)args;
  __shared__ float red[REDN];
  __shared__ float win[STG ? STG : 1];
  CglKL L = cgl_conv_args();
  CglKP P = &L->p[0];
  const int lanes = C4T ? C4T : (P->Cin >> 2), slots = 256 / lanes;
  const int Cin = 4 * lanes, Tx = P->Tx, T = P->Ty * P->Tx;
  const int q4 = threadIdx.x & (lanes - 1), slot = threadIdx.x / lanes;
  const int XH = XHT ? XHT : P->XH, XW = XWT ? XWT : P->XW, OH = P->OH, OW = P->OW;
  const int hw = XH * XW;
  const long Min = (long)(P->M / (OH * OW)) * hw;
  const int splits = P->splits;
  const long qb = (blockIdx.x * Min) / splits, qe = ((blockIdx.x + 1) * Min) / splits;
  f32x4 acc[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 isc = {0.f, 0.f, 0.f, 0.f}, ish = isc;
  const float in_sl = BNIN ? cgl_bnin_slope(L) : 0.f;       // (in registers: see the halo staging)
  if constexpr (BNIN) {
    isc = *(gcf4p)(L->in_coef + (long)L->in_g0 * Cin + 4 * q4);
    ish = *(gcf4p)(L->in_coef + (long)(L->in_groups + L->in_g0) * Cin + 4 * q4);
  }
  const float* __restrict__ dY = P->Y;
  const long wb = qb - OW - 1;
  if (STG) {
    const long wl = (qe - qb) + 2 * OW + 2, Mo = P->M;
    for (int i = threadIdx.x; i < wl; i += 256) {
      const long lin = wb + i;
      const float v = gld(dY + min(max(lin, 0L), Mo - 1));
      win[i] = (lin >= 0 && lin < Mo) ? v : 0.f;
    }
    __syncthreads();
  }
  // CGL_N1T_PX input pixels per step: every pixel's loads (1 float4 + T gathers each) are in flight
  // before the first FMA; the pixels of a step are accumulated in order (fixed summation order)
  for (long q0 = qb + slot; q0 < qe; q0 += CGL_N1T_PX * slots) {
    f32x4 x[CGL_N1T_PX];
    float d[CGL_N1T_PX][16];
#pragma unroll
    for (int u = 0; u < CGL_N1T_PX; ++u) {
      const long qq = min(q0 + u * slots, qe - 1);
      const int img = (int)(qq / hw);
      const int r = (int)(qq - (long)img * hw);
      const int iy = r / XW, ix = r - iy * XW;
      x[u] = *(gcf4p)(P->X + qq * Cin + 4 * q4);
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        if (t < T) {
          const int ty = t / Tx, tx = t - ty * Tx;
          const int oy = iy - P->dy[ty], ox = ix - P->dx[tx];
          const bool ok = (unsigned)oy < (unsigned)OH && (unsigned)ox < (unsigned)OW && q0 + u * slots < qe;
          float dv;
          if (STG)
            dv = win[(int)(qq - wb) - P->dy[ty] * OW - P->dx[tx]];
          else
            dv = gld(dY + (((long)img * P->YH + min(max(oy, 0), OH - 1)) * P->YW + min(max(ox, 0), OW - 1)) *
                              P->ldy);
          d[u][t] = ok ? dv : 0.f;
        }
      }
    }
    if constexpr (BNIN) {
#pragma unroll
      for (int u = 0; u < CGL_N1T_PX; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float w = fmaf(x[u][e], isc[e], ish[e]);
          w = fmaxf(w, w * in_sl);
          x[u][e] = w;
        }
    }
#pragma unroll
    for (int u = 0; u < CGL_N1T_PX; ++u)
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        if (t < T) {
          acc[t][0] = fmaf(x[u][0], d[u][t], acc[t][0]);
          acc[t][1] = fmaf(x[u][1], d[u][t], acc[t][1]);
          acc[t][2] = fmaf(x[u][2], d[u][t], acc[t][2]);
          acc[t][3] = fmaf(x[u][3], d[u][t], acc[t][3]);
        }
      }
  }
  const int K = T * Cin;
#pragma unroll
  for (int t = 0; t < 16; ++t)
    if (t < T) *(f32x4*)&red[slot * K + t * Cin + 4 * q4] = acc[t];
  __syncthreads();
  for (int k = threadIdx.x; k < K; k += 256) {
    float v = 0.f;
    for (int sl = 0; sl < slots; ++sl) v += red[sl * K + k];
    gst(P->part + (long)blockIdx.x * P->Kp + k, v);
  }
}

// Input gradient of a stride-1 3x3 one-output-channel convolution (Conv2d(64, 1, 3, 1, 1) + Tanh,
// model/lsgan.py:19-20): dX(i, c) = sum_t dY(i - d_t) W[0][c][t], 9 FMAs per written element, so the
// op is a write stream of dX.  C4 = Cin / 4 lanes own one input pixel (a float4 of channels: a wave's
// stores cover 64 / C4 consecutive pixels, fully coalesced); the lane's 9 weight quads are read from
// the reference's OIHW W once (no packing launch) and stay in registers; the 9 dY scalars are
// broadcast reads of a 4 KB image (L1 / L2 hits).  Taps are summed in (ky, kx) order.
#define CGL_BN1_PPT 8
// ST: also the next BatchNorm2d backward's per-chunk partials (cgl_chan_reduce4 mode 1 of dX, fused): a workgroup's
// CGL_BN1_PPT x 16 pixels are one 128-row chunk, and lane (pixel slot rl, channel quad q) holds rows rl + 16 k in k
// order -- the very rows, order and lane-then-slot sums of cgl_chan_reduce4 with R = 128, so the partials are
// bitwise the ones cgl_bn2d_bwd computes from the stored dX.
struct CglN1Stats {
  const float* X;            // [npix][4 C4] the BatchNorm's input y (pre-normalisation)
  const float* post;         // LeakyReLU'(post), or null
  const float* psc; int psc_ld;   // or LeakyReLU' from the sign of fmaf(y, scale, shift)
  const float* mean;         // [groups][4 C4]
  float slope;
  int gr;                    // rows per group (a multiple of 128)
  double* part;              // [npix / 128][4 C4][2]
};
template <int C4, bool ST = false>
__global__ __launch_bounds__(256) void cgl_conv_bwd_n1(const float* __restrict__ dY, const float* __restrict__ W,
                                                       float* __restrict__ dX, int npix, int H, int Wd, CglN1Stats st) {
  const int q = threadIdx.x & (C4 - 1);
  f32x4 w[9];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) w[t][j] = gld(W + (4 * q + j) * 9 + t);
  double x0[4] = {0.0, 0.0, 0.0, 0.0}, x1[4] = {0.0, 0.0, 0.0, 0.0};
  f32x4 mu = {}, ps = {}, ph = {};
  float slope = 0.f;
  if constexpr (ST) {
    const int r0 = blockIdx.x * (CGL_BN1_PPT * (256 / C4));
    mu = *(gcf4p)(st.mean + (long)(r0 / st.gr) * (4 * C4) + 4 * q);
    if (st.psc) {
      ps = *(gcf4p)(st.psc + 4 * q);
      ph = *(gcf4p)(st.psc + st.psc_ld + 4 * q);
    }
    slope = st.slope;
  }
  // the statistics' y values of all CGL_BN1_PPT pixels in flight before the first dY gather
  f32x4 xs[ST ? CGL_BN1_PPT : 1];
  if constexpr (ST) {
#pragma unroll
    for (int k = 0; k < CGL_BN1_PPT; ++k)
      xs[k] = *(gcf4p)(st.X + ((long)((blockIdx.x * CGL_BN1_PPT + k) * (256 / C4) + (int)threadIdx.x / C4)) * (4 * C4) +
                       4 * q);
  }
  // CGL_BN1_PPT pixels per lane group (the weight loads amortised over them), consecutive groups of a
  // workgroup on consecutive pixels
  constexpr int kUnroll = ST ? CGL_BN1_PPT : 2;
#pragma unroll kUnroll
  for (int k = 0; k < CGL_BN1_PPT; ++k) {
  const int p = (blockIdx.x * CGL_BN1_PPT + k) * (256 / C4) + (int)threadIdx.x / C4;
  const int pc = min(p, npix - 1);
  const int hw = H * Wd;
  const int img = pc / hw, r = pc - img * hw;
  const int y = r / Wd, x = r - y * Wd;
  const float* __restrict__ d = dY + (long)img * hw;
  float dv[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int oy = y + 1 - t / 3, ox = x + 1 - t % 3;
    const bool ok = (unsigned)oy < (unsigned)H && (unsigned)ox < (unsigned)Wd;
    const float v = gld(d + min(max(oy, 0), H - 1) * Wd + min(max(ox, 0), Wd - 1));
    dv[t] = ok ? v : 0.f;
  }
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    acc[0] = fmaf(dv[t], w[t][0], acc[0]);
    acc[1] = fmaf(dv[t], w[t][1], acc[1]);
    acc[2] = fmaf(dv[t], w[t][2], acc[2]);
    acc[3] = fmaf(dv[t], w[t][3], acc[3]);
  }
  if (p < npix) *(gf4p)(dX + (long)p * (4 * C4) + 4 * q) = acc;
  if constexpr (ST) {     // (the launch covers whole chunks: every p < npix)
    const long o = (long)p * (4 * C4) + 4 * q;
    const f32x4 xv = xs[ST ? k : 0];
    f32x4 g = acc;
    if (st.psc) {
#pragma unroll
      for (int j = 0; j < 4; ++j) g[j] = fmaf(xv[j], ps[j], ph[j]) > 0.f ? g[j] : g[j] * slope;
    } else if (st.post) {
      const f32x4 pv = *(gcf4p)(st.post + o);
#pragma unroll
      for (int j = 0; j < 4; ++j) g[j] = pv[j] > 0.f ? g[j] : g[j] * slope;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x0[j] += (double)g[j];
      x1[j] += (double)(g[j] * (xv[j] - mu[j]));
    }
  }
  }
  if constexpr (ST) {
    __shared__ double s0[1024], s1[1024];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s0[threadIdx.x * 4 + j] = x0[j];
      s1[threadIdx.x * 4 + j] = x1[j];
    }
    __syncthreads();
    if ((int)threadIdx.x < C4) {
      constexpr int rp = 256 / C4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        double t0 = 0.0, t1 = 0.0;
        for (int r = 0; r < rp; ++r) {
          t0 += s0[(r * C4 + q) * 4 + j];
          t1 += s1[(r * C4 + q) * 4 + j];
        }
        st.part[((long)blockIdx.x * (4 * C4) + 4 * q + j) * 2] = t0;
        st.part[((long)blockIdx.x * (4 * C4) + 4 * q + j) * 2 + 1] = t1;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// One-input-channel 3x3 convolutions on the vector ALUs (the discriminator's Conv2d(1, 16, 3, 2, 1),
// model/lsgan.py:78 on the 32x32 image): 9 MACs per output element are far too few for an MFMA
// tile (the implicit GEMM decoded its k index per element and ran 4-6x slower than this).
//   forward: one thread per output pixel, the 9 input taps in registers, the weights in LDS
//   (broadcast reads), bias + activation + Dropout2d scale fused, cout floats stored contiguously;
//   weight gradient: thread (channel, pixel lane) accumulates its channel's 9 taps + bias over a
//   pixel slice, the block's lanes are summed through LDS in a fixed order into per-block partials,
//   and cgl_conv_c1_wgrad_fin sums the blocks in order (double) into dW [cout][1][3][3] and db.
struct CglC1Args {
  const float* X; const float* W; int wst;   // weights: row co at W + co * wst, 9 taps
  const float* bias; float* Y; const float* drop;
  const float* dY; float* part; float* dW; float* db;
  int n, h, w, ho, wo, cout, stride, act, nblk, chunk;
  float slope;
  // weight gradient only: dY is the gradient at the block's OUTPUT -- the LeakyReLU (post = its output) and
  // Dropout2d (drop [n][cout]) backward are applied per loaded value in cgl_act_drop_bwd's order (bitwise)
  const float* post;
};

__global__ __launch_bounds__(256) void cgl_conv_c1_fwd(CglC1Args a) {
  __shared__ float sw[64 * 9], sb[64];
  const int tid = threadIdx.x, cout = a.cout;
  for (int e = tid; e < cout * 9; e += 256) sw[e] = gld(a.W + (e / 9) * a.wst + e % 9);
  if (tid < cout) sb[tid] = a.bias ? gld(a.bias + tid) : 0.f;
  __syncthreads();
  const int hw = a.ho * a.wo;
  const long p = (long)blockIdx.x * 256 + tid;
  if (p >= (long)a.n * hw) return;
  const int img = (int)(p / hw), r = (int)(p - (long)img * hw), oy = r / a.wo, ox = r - oy * a.wo;
  float xv[9];
  const float* xi = a.X + (long)img * a.h * a.w;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int iy = oy * a.stride + t / 3 - 1, ix = ox * a.stride + t % 3 - 1;
    const bool ok = (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w;
    const float v = gld(xi + min(max(iy, 0), a.h - 1) * a.w + min(max(ix, 0), a.w - 1));
    xv[t] = ok ? v : 0.f;
  }
  for (int c4 = 0; c4 < cout; c4 += 4) {
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float v = sb[c4 + j];
#pragma unroll
      for (int t = 0; t < 9; ++t) v = fmaf(xv[t], sw[(c4 + j) * 9 + t], v);
      if (a.act == CGL_EPI_ACT_LEAKY) v = v > 0.f ? v : v * a.slope;
      o[j] = v;
    }
    if (a.drop) {
      const f32x4 dm = *(gcf4p)(a.drop + (long)img * cout + c4);
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] *= dm[j];
    }
    *(gf4p)(a.Y + p * cout + c4) = o;
  }
}

#define CGL_C1_PPT 8
__global__ __launch_bounds__(256) void cgl_conv_c1_wgrad(CglC1Args a) {
  __shared__ float red[256 * 10];
  const int tid = threadIdx.x, cout = a.cout, lanes = 256 / cout;
  const int co = tid % cout, lj = tid / cout;
  const int hw = a.ho * a.wo;
  const long npix = (long)a.n * hw;
  const long p0 = (long)blockIdx.x * a.chunk, p1 = min(p0 + a.chunk, npix);
  float acc[10];
#pragma unroll
  for (int t = 0; t < 10; ++t) acc[t] = 0.f;
  // CGL_C1_PPT pixels per thread per pass, every load of the pass issued before the first use
  for (long pb = p0 + lj; pb < p1; pb += (long)CGL_C1_PPT * lanes) {
    float dy[CGL_C1_PPT], xv[CGL_C1_PPT][9];
#pragma unroll
    for (int u = 0; u < CGL_C1_PPT; ++u) {
      const long p = min(pb + (long)u * lanes, p1 - 1);
      const int img = (int)(p / hw), r = (int)(p - (long)img * hw), oy = r / a.wo, ox = r - oy * a.wo;
      float d = gld(a.dY + p * cout + co);
      if (a.post) d = gld(a.post + p * cout + co) > 0.f ? d : d * a.slope;
      if (a.drop) d *= gld(a.drop + (long)img * cout + co);
      dy[u] = pb + (long)u * lanes < p1 ? d : 0.f;
      const float* xi = a.X + (long)img * a.h * a.w;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int iy = oy * a.stride + t / 3 - 1, ix = ox * a.stride + t % 3 - 1;
        const bool ok = (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w;
        const float v = gld(xi + min(max(iy, 0), a.h - 1) * a.w + min(max(ix, 0), a.w - 1));
        xv[u][t] = ok ? v : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < CGL_C1_PPT; ++u) {
#pragma unroll
      for (int t = 0; t < 9; ++t) acc[t] = fmaf(dy[u], xv[u][t], acc[t]);
      acc[9] += dy[u];
    }
  }
#pragma unroll
  for (int t = 0; t < 10; ++t) red[t * 256 + tid] = acc[t];
  __syncthreads();
  if (tid < cout * 10) {        // (channel, tap) = (tid % cout, tid / cout): lanes summed in order
    const int c = tid % cout, t = tid / cout;
    float v = 0.f;
    for (int l = 0; l < lanes; ++l) v += red[t * 256 + l * cout + c];
    a.part[(long)blockIdx.x * cout * 10 + t * cout + c] = v;
  }
}

__device__ __forceinline__ double cgl_block_sum_d(double x, double* red);

// one workgroup per (tap, channel) output: blocks b = thread, thread + 256, ... summed in order,
// then the fixed-order block sum
template <class CA>
__device__ __forceinline__ void cgl_conv_c1_wgrad_fin_at(const CA& a, int o, double* red) {
  const int cout = a.cout, tid = threadIdx.x;
  double v = 0.0;
  for (int b = tid; b < a.nblk; b += 256) v += (double)gld(a.part + (long)b * cout * 10 + o);
  v = cgl_block_sum_d(v, red);
  if (tid == 0) {
    const int c = o % cout, t = o / cout;
    if (t < 9) gst(a.dW + c * 9 + t, (float)v);
    else if (a.db) gst(a.db + c, (float)v);
  }
}

__global__ __launch_bounds__(256) void cgl_conv_c1_wgrad_fin(CglC1Args a) {
  __shared__ double red[4];
  cgl_conv_c1_wgrad_fin_at(a, (int)blockIdx.x, red);
}

// ------------------------------------------------------------------------------------------
// Weight packing: Wp_p[n][k] = sum over the kernel taps combined into packed tap t of W (OIHW),
// (co, ci) = (n, c) for a forward problem, (c, n) for an input-gradient problem (transpose);
// zero for k >= K (row padding to a multiple of 16).
struct CglPackArgs {
  const float* W;            // [cout][cin][ks][ks]
  int cout, cin, transpose, np, ks;
  float* dst[CGL_CONV_MAXP];
  int N[CGL_CONV_MAXP], Kp[CGL_CONV_MAXP], Cg[CGL_CONV_MAXP], Tx[CGL_CONV_MAXP], T[CGL_CONV_MAXP];
  int ym[CGL_CONV_MAXP][4], xm[CGL_CONV_MAXP][4];
  int begin[CGL_CONV_MAXP + 1];  // element offsets of each problem in the grid
};

__global__ __launch_bounds__(256) void cgl_conv_pack(CglPackArgs a) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= a.begin[a.np]) return;
  int p = 0;
  for (int q = 1; q < a.np; ++q)
    if (e >= a.begin[q]) p = q;
  const int local = e - a.begin[p];
  const int Kp = a.Kp[p], Cg = a.Cg[p];
  const int n = local / Kp, k = local - n * Kp;
  float v = 0.f;
  if (k < a.T[p] * Cg) {
    const int t = k / Cg, c = k - t * Cg;
    const int ty = t / a.Tx[p], tx = t - ty * a.Tx[p];
    const int co = a.transpose ? c : n, ci = a.transpose ? n : c;
    const int ks = a.ks;
    const float* w = a.W + ((long)co * a.cin + ci) * ks * ks;
    const int ymk = a.ym[p][ty], xmk = a.xm[p][tx];
    for (int kh = 0; kh < ks; ++kh) {
      if (!((ymk >> kh) & 1)) continue;
      for (int kw = 0; kw < ks; ++kw)
        if ((xmk >> kw) & 1) v += gld(w + kh * ks + kw);
    }
  }
  gst(a.dst[p] + local, v);
}

// Multi-op weight pack: every packed problem of several (layer, direction) pairs -- a whole model's
// forward and input-gradient operands -- in ONE launch, so that a training round re-packs each
// model once per parameter update instead of once per convolution call.  Each job starts on a
// block boundary, so the job lookup is uniform (scalar) per block.
#define CGL_PACKM_MAXJ 48
struct CglPackJobK {
  const float* W;            // [cout][cin][ks][ks]
  float* dst;                // packed [N][Kp]
  int cout, cin, transpose, ks, N, Kp, Cg, Tx, T;
  int tapm;                  // ym[ty] in bits 4 ty .. 4 ty + 3, xm[tx] in bits 16 + 4 tx ..
  int blk_begin;
};
struct CglPackMultiArgs {
  int nj, pad;
  CglPackJobK j[CGL_PACKM_MAXJ];
};

__device__ __forceinline__ void cgl_conv_pack_at(const CGL_AS4 CglPackMultiArgs* A, int b) {
  int q = 0;
  for (int i = 1; i < A->nj; ++i)
    if (b >= A->j[i].blk_begin) q = i;
  const CGL_AS4 CglPackJobK* J = &A->j[q];
  const int Kp = J->Kp, Cg = J->Cg;
  const int local = (b - J->blk_begin) * 256 + (int)threadIdx.x;
  if (local >= J->N * Kp) return;
  const int n = local / Kp, k = local - n * Kp;
  float v = 0.f;
  if (k < J->T * Cg) {
    const int t = k / Cg, c = k - t * Cg;
    const int ty = t / J->Tx, tx = t - ty * J->Tx;
    const int co = J->transpose ? c : n, ci = J->transpose ? n : c;
    const int ks = J->ks;
    const float* w = J->W + ((long)co * J->cin + ci) * ks * ks;
    const int ymk = (J->tapm >> (4 * ty)) & 15, xmk = (J->tapm >> (16 + 4 * tx)) & 15;
    if (ks == 3) {
      // every tap's weight loaded up front (one memory round trip, not one per combined tap), then summed in the
      // same (kh, kw) order over the combined taps: the same value
      float wv[9];
#pragma unroll
      for (int i = 0; i < 9; ++i) wv[i] = gld(w + i);
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
          if (((ymk >> kh) & 1) && ((xmk >> kw) & 1)) v += wv[kh * 3 + kw];
    } else {
      for (int kh = 0; kh < ks; ++kh) {
        if (!((ymk >> kh) & 1)) continue;
        for (int kw = 0; kw < ks; ++kw)
          if ((xmk >> kw) & 1) v += gld(w + kh * ks + kw);
      }
    }
  }
  gst(J->dst + local, v);
}

__global__ __launch_bounds__(256) void cgl_conv_pack_multi(CglPackMultiArgs) {
  typedef const CGL_AS4 CglPackMultiArgs* KA;
  cgl_conv_pack_at((KA)__builtin_amdgcn_kernarg_segment_ptr(), blockIdx.x);
}

// Weight-gradient reduction: dW[co][ci][kh][kw] = sum over problems, taps containing (kh, kw) and
// splits of the partial tiles.  A block covers EB consecutive elements
// e = ((co * ks + kh) * ks + kw) * cin + ci (consecutive ci: coalesced partial reads) x SG
// split-groups (split-group g sums splits g, g + SG, ... in order, 8 loads in flight); the SG
// partial sums are combined through LDS in a fixed order (deterministic).
struct CglWgradReduceArgs {
  float* dW;
  float* db;                 // bias gradient from the partials' column K (or null)
  int cout, cin, np, ks, EB, SG;
  int wblocks;               // blocks of the dW elements; the db blocks follow
  int K[CGL_CONV_MAXP];
  const float* part[CGL_CONV_MAXP];
  int Kp[CGL_CONV_MAXP], splits[CGL_CONV_MAXP], Tx[CGL_CONV_MAXP], Ty[CGL_CONV_MAXP];
  int ym[CGL_CONV_MAXP][4], xm[CGL_CONV_MAXP][4];
};

// block bid of a weight gradient's fixed-order split reduction (cgl_conv_wgrad_reduce, cgl_conv_wgrad_reduce_multi);
// RA: the by-value argument or its copy inside the multi-launch's kernarg block; red: 256 doubles of LDS
template <class RA>
__device__ __forceinline__ void cgl_conv_wgrad_reduce_at(const RA& a, int bid, double* red) {
  const int EB = a.EB, SG = a.SG;
  const int el = threadIdx.x % EB, sg = threadIdx.x / EB;
  const int e = bid * EB + el;
  const int cin = a.cin, ks = a.ks;
  const int E = a.cout * ks * ks * cin;
  if (a.db && bid >= a.wblocks) {   // uniform per block
    // bias gradient: db[co] = sum over problems and splits of part[s][co][K]
    const int eb = (bid - a.wblocks) * EB + el;
    const int co = min(eb, a.cout - 1);
    double acc = 0.0;
    for (int p = 0; p < a.np; ++p) {
      const int S = a.splits[p];
      const long sstride = (long)a.cout * a.Kp[p];
      const float* src = a.part[p] + (long)co * a.Kp[p] + a.K[p];
      for (int s0 = sg; s0 < S; s0 += 8 * SG) {
        float v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = gld(src + (long)min(s0 + i * SG, S - 1) * sstride);
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (s0 + i * SG < S) acc += (double)v[i];
      }
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    if (sg == 0 && eb < a.cout) {
      double t = 0.0;
      for (int g = 0; g < SG; ++g) t += red[g * EB + el];
      gst(a.db + eb, (float)t);
    }
    return;
  }
  const int ee = min(e, E - 1);
  const int ci = ee % cin;
  const int rest = ee / cin;
  const int kw = rest % ks, kh = (rest / ks) % ks, co = rest / (ks * ks);
  double acc = 0.0;
  for (int p = 0; p < a.np; ++p) {
    const int Kp = a.Kp[p], Tx = a.Tx[p], Ty = a.Ty[p], S = a.splits[p];
    const long sstride = (long)a.cout * Kp;
    for (int ty = 0; ty < Ty; ++ty) {
      if (!((a.ym[p][ty] >> kh) & 1)) continue;
      for (int tx = 0; tx < Tx; ++tx) {
        if (!((a.xm[p][tx] >> kw) & 1)) continue;
        const float* src = a.part[p] + (long)co * Kp + (ty * Tx + tx) * cin + ci;
        for (int s0 = sg; s0 < S; s0 += 8 * SG) {
          float v[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) v[i] = gld(src + (long)min(s0 + i * SG, S - 1) * sstride);
#pragma unroll
          for (int i = 0; i < 8; ++i)
            if (s0 + i * SG < S) acc += (double)v[i];
        }
      }
    }
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  if (sg == 0 && e < E) {
    double t = 0.0;
    for (int g = 0; g < SG; ++g) t += red[g * EB + el];
    gst(a.dW + ((long)co * cin + ci) * ks * ks + kh * ks + kw, (float)t);
  }
}

__global__ __launch_bounds__(256) void cgl_conv_wgrad_reduce(CglWgradReduceArgs a) {
  __shared__ double red[256];
  cgl_conv_wgrad_reduce_at(a, (int)blockIdx.x, red);
}


// ------------------------------------------------------------------------------------------
// Per-channel reductions over an NHWC tensor [rows][C] (C a power of two <= 256), one chunk of R
// rows per workgroup, double accumulation, fixed order:
//   mode 0  {sum x, M2 about the chunk mean}                            (BatchNorm2d statistics)
//   mode 1  {sum g, sum g (x - mean_group)},  g = dY * leaky'(post)      (BatchNorm2d backward)
//   mode 2  {sum x, 0}                                                  (bias gradient)
struct CglChanArgs {
  const float* X; int rows, C, R, mode, hw, gr;
  const float* dY; const float* post; float slope;
  const float* mean;         // [groups][C] (mode 1)
  double* part;              // [nchunks][C][2]
  const int* nv;             // mode 0: only rows < *nv * hw of the first group (rows < gr) count, or null
  // mode 1 without the post-activation tensor: LeakyReLU'(post) from the sign of the forward's own
  // fmaf(x, scale, shift) (scale = psc[c], shift = psc[psc_ld + c]) -- post > 0 exactly when that value is
  // (slope > 0), so the gradient is bitwise the one read from post, and post's bytes are not read
  const float* psc; int psc_ld;
};

// rows of the first BatchNorm group that carry data: a short real call (DataLoader's short final batch)
// holds *nv real images, the rest of its gr rows are padding; null = the whole group
__device__ __forceinline__ int cgl_nv_rows(const int* nv, int hw, int gr) {
  return nv ? min(gldi(nv) * hw, gr) : gr;
}

__global__ __launch_bounds__(256) void cgl_chan_reduce(CglChanArgs a) {
  __shared__ double s0[256], s1[256];
  const int C = a.C, rp = 256 / C;
  const int c = threadIdx.x % C, rl = threadIdx.x / C;
  const int r0 = blockIdx.x * a.R;
  int r1 = min(r0 + a.R, a.rows);
  if (a.mode == 0 && a.nv && r0 < a.gr) r1 = max(r0, min(r1, cgl_nv_rows(a.nv, a.hw, a.gr)));
  double x0 = 0.0, x1 = 0.0;
  // rows r0 + rl + rp * i, issued 8 at a time (independent loads in flight), summed in order
  if (a.mode == 1) {
    const float mu = gld(a.mean + (long)(r0 / a.gr) * C + c);
    for (int rb = r0 + rl; rb < r1; rb += 8 * rp) {
      float g[8], xv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = min(rb + i * rp, r1 - 1);
        const long o = (long)r * C + c;
        g[i] = gld(a.dY + o);
        if (a.psc) g[i] = fmaf(xv[i], a.psc[c], a.psc[a.psc_ld + c]) > 0.f ? g[i] : g[i] * a.slope;
        else if (a.post) g[i] = gld(a.post + o) > 0.f ? g[i] : g[i] * a.slope;
        xv[i] = gld(a.X + o);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (rb + i * rp < r1) {
          x0 += (double)g[i];
          x1 += (double)(g[i] * (xv[i] - mu));
        }
    }
  } else {
    for (int rb = r0 + rl; rb < r1; rb += 8 * rp) {
      float xv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) xv[i] = gld(a.X + (long)min(rb + i * rp, r1 - 1) * C + c);
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (rb + i * rp < r1) x0 += (double)xv[i];
    }
  }
  s0[threadIdx.x] = x0;
  s1[threadIdx.x] = x1;
  __syncthreads();
  if (a.mode == 0) {
    if (rl == 0) {
      double t = 0.0;
      for (int q = 0; q < rp; ++q) t += s0[q * C + c];
      s0[c] = t;
    }
    __syncthreads();
    const double mean = s0[c] / max(r1 - r0, 1);
    double m2 = 0.0;
    for (int rb = r0 + rl; rb < r1; rb += 8 * rp) {
      float xv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) xv[i] = gld(a.X + (long)min(rb + i * rp, r1 - 1) * C + c);
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (rb + i * rp < r1) {
          const double d = (double)xv[i] - mean;
          m2 += d * d;
        }
    }
    __syncthreads();
    s1[threadIdx.x] = m2;
    __syncthreads();
    if (rl == 0) {
      double t = 0.0;
      for (int q = 0; q < rp; ++q) t += s1[q * C + c];
      a.part[((long)blockIdx.x * C + c) * 2] = s0[c];
      a.part[((long)blockIdx.x * C + c) * 2 + 1] = t;
    }
    return;
  }
  if (rl == 0) {
    double t0 = 0.0, t1 = 0.0;
    for (int q = 0; q < rp; ++q) {
      t0 += s0[q * C + c];
      t1 += s1[q * C + c];
    }
    a.part[((long)blockIdx.x * C + c) * 2] = t0;
    a.part[((long)blockIdx.x * C + c) * 2 + 1] = t1;
  }
}

// 16-byte variant of cgl_chan_reduce for C % 4 == 0 (every BatchNorm2d of model/lsgan.py): a lane owns
// a float4 of channels, so each row of a wave's load is one 16-byte access per lane (4x fewer vector
// memory instructions than the per-channel lanes above) and 8 rows x 16 B are in flight per lane.
// Same outputs (double partials per chunk and channel; rows summed per lane in row order, lanes in
// a fixed order).
__global__ __launch_bounds__(256) void cgl_chan_reduce4(CglChanArgs a) {
  __shared__ double s0[1024], s1[1024], tot[256];
  const int C = a.C, CW = C >> 2, rp = 256 / CW;
  const int cs = threadIdx.x % CW, rl = threadIdx.x / CW, c = 4 * cs;
  const int r0 = blockIdx.x * a.R;
  int r1 = min(r0 + a.R, a.rows);
  if (a.mode == 0 && a.nv && r0 < a.gr) r1 = max(r0, min(r1, cgl_nv_rows(a.nv, a.hw, a.gr)));
  double x0[4] = {0.0, 0.0, 0.0, 0.0}, x1[4] = {0.0, 0.0, 0.0, 0.0};
  if (a.mode == 1) {
    const f32x4 mu = *(gcf4p)(a.mean + (long)(r0 / a.gr) * C + c);
    const f32x4 ps = a.psc ? *(gcf4p)(a.psc + c) : mu, ph = a.psc ? *(gcf4p)(a.psc + a.psc_ld + c) : mu;
    for (int rb = r0 + rl; rb < r1; rb += 8 * rp) {
      f32x4 g[8], xv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const long o = (long)min(rb + i * rp, r1 - 1) * C + c;
        g[i] = *(gcf4p)(a.dY + o);
        xv[i] = *(gcf4p)(a.X + o);
        if (a.psc) {
#pragma unroll
          for (int j = 0; j < 4; ++j) g[i][j] = fmaf(xv[i][j], ps[j], ph[j]) > 0.f ? g[i][j] : g[i][j] * a.slope;
        } else if (a.post) {
          const f32x4 p = *(gcf4p)(a.post + o);
#pragma unroll
          for (int j = 0; j < 4; ++j) g[i][j] = p[j] > 0.f ? g[i][j] : g[i][j] * a.slope;
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (rb + i * rp < r1) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            x0[j] += (double)g[i][j];
            x1[j] += (double)(g[i][j] * (xv[i][j] - mu[j]));
          }
        }
    }
  } else {
    for (int rb = r0 + rl; rb < r1; rb += 8 * rp) {
      f32x4 xv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) xv[i] = *(gcf4p)(a.X + (long)min(rb + i * rp, r1 - 1) * C + c);
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (rb + i * rp < r1) {
#pragma unroll
          for (int j = 0; j < 4; ++j) x0[j] += (double)xv[i][j];
        }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    s0[threadIdx.x * 4 + j] = x0[j];
    s1[threadIdx.x * 4 + j] = x1[j];
  }
  __syncthreads();
  if (a.mode == 0) {
    if (rl == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        double t = 0.0;
        for (int q = 0; q < rp; ++q) t += s0[(q * CW + cs) * 4 + j];
        tot[c + j] = t;
      }
    }
    __syncthreads();
    double mean[4], m2[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int j = 0; j < 4; ++j) mean[j] = tot[c + j] / max(r1 - r0, 1);
    for (int rb = r0 + rl; rb < r1; rb += 8 * rp) {
      f32x4 xv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) xv[i] = *(gcf4p)(a.X + (long)min(rb + i * rp, r1 - 1) * C + c);
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (rb + i * rp < r1) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const double d = (double)xv[i][j] - mean[j];
            m2[j] += d * d;
          }
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) s1[threadIdx.x * 4 + j] = m2[j];
    __syncthreads();
    if (rl == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        double t = 0.0;
        for (int q = 0; q < rp; ++q) t += s1[(q * CW + cs) * 4 + j];
        a.part[((long)blockIdx.x * C + c + j) * 2] = tot[c + j];
        a.part[((long)blockIdx.x * C + c + j) * 2 + 1] = t;
      }
    }
    return;
  }
  if (rl == 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      double t0 = 0.0, t1 = 0.0;
      for (int q = 0; q < rp; ++q) {
        t0 += s0[(q * CW + cs) * 4 + j];
        t1 += s1[(q * CW + cs) * 4 + j];
      }
      a.part[((long)blockIdx.x * C + c + j) * 2] = t0;
      a.part[((long)blockIdx.x * C + c + j) * 2 + 1] = t1;
    }
  }
}

// launch the 16-byte variant when every operand allows it
inline void launch_chan_reduce(const CglChanArgs& a, int nch, hipStream_t s) {
  auto ok = [](const void* p) { return p == nullptr || ((uintptr_t)p & 15) == 0; };
  if (a.C % 4 == 0 && a.C >= 4 && a.C <= 256 && 256 % (a.C / 4) == 0 && ok(a.X) && ok(a.dY) && ok(a.post) &&
      ok(a.mean) && !getenv("CGL_CHAN_SCALAR"))
    hipLaunchKernelGGL(cgl_chan_reduce4, dim3(nch), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(cgl_chan_reduce, dim3(nch), dim3(256), 0, s, a);
}

// Column sums of X [rows][C] per chunk of R rows (any C): part[chunk][c][0] (double); 8 loads in
// flight per thread, summed in row order.
__global__ __launch_bounds__(256) void cgl_colsum_k(const float* X, int rows, int C, int R, double* part) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const int r0 = blockIdx.y * R, r1 = min(r0 + R, rows);
  double t = 0.0;
  for (int rb = r0; rb < r1; rb += 8) {
    float xv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) xv[i] = gld(X + (long)min(rb + i, r1 - 1) * C + c);
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (rb + i < r1) t += (double)xv[i];
  }
  part[((long)blockIdx.y * C + c) * 2] = t;
  part[((long)blockIdx.y * C + c) * 2 + 1] = 0.0;
}

// BatchNorm2d finalize: ONE WORKGROUP PER CHANNEL, threads over the chunk partials (thread t takes
// chunks t, t + 256, ... in order, then a fixed xor-tree in each wave and the 4 wave sums in wave
// order: deterministic), groups in the reference's call order.
//   fwd (mode 0): mean / biased var per group from the chunk partials (Chan), save_mean / invstd,
//                 scale = invstd * gamma, shift = beta - mean * scale, running stats (momentum,
//                 unbiased variance) group by group; eval: the same from running stats.
//   bwd (mode 1): per group gm = S / n, k = D invstd^2 / n; dgamma = sum_g D invstd, dbeta = sum_g S.
//   bias (mode 2): out = sum of every chunk.
struct CglBnFinArgs {
  const double* part; int C, groups, chunks_per_group, R, gr, mode, train;
  const float* gamma; const float* beta;
  double eps, momentum;
  float* run_mean; float* run_var;
  float* save_mean; float* save_invstd;     // [groups][C]
  float* coef0; float* coef1;               // [groups][C]: fwd scale, shift; bwd gm, k
  float* dgamma; float* dbeta;              // bwd, or bias out (mode 2: dgamma)
  int nocache;                              // A/B switch: stream the partials twice (CGL_FIN_NOCACHE)
  // a short first call (the D step's real call on DataLoader's short final batch): only its first *nv images
  // (hw rows each) carry data -- group 0 counts nv * hw rows, and chunk q of it min(max(nv hw - q R, 0), R)
  const int* nv; int hw;
};

// rows of group g and of chunk q of it (cgl_nv_rows for the short first call)
__device__ __forceinline__ int cgl_fin_rows(const CglBnFinArgs& a, int g) {
  return g == 0 ? cgl_nv_rows(a.nv, a.hw, a.gr) : a.gr;
}
__device__ __forceinline__ int cgl_fin_chunk_rows(int n, int q, int R) { return min(max(n - q * R, 0), R); }

__device__ __forceinline__ double cgl_wave_sum_d(double x) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

// sum over the 256 threads of a workgroup, returned to every thread (every thread must call it)
__device__ __forceinline__ double cgl_block_sum_d(double x, double* red) {
  x = cgl_wave_sum_d(x);
  __syncthreads();                       // red[] free (a previous call may still be reading it)
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = x;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// sum over chunks q = lane, lane + 256, ... < cnt of f(part pair at chunk q0 + q) -- 8 independent
// 16-byte loads in flight per thread, accumulated in chunk order (the per-thread order is fixed)
// (fn(pair, q): q = the chunk's index within its group, qbase = that of chunk q0)
template <class Fn>
__device__ __forceinline__ double cgl_fin_sum(const double* part, long q0, int cnt, int C, int c, int lane, Fn fn,
                                              int qbase = 0) {
  typedef double f64x2 __attribute__((ext_vector_type(2)));
  typedef const CGL_GLOBAL f64x2* gcd2p;
  double t = 0.0;
  for (int qb = lane; qb < cnt; qb += 8 * 256) {
    f64x2 v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = *(gcd2p)(part + ((q0 + min(qb + 256 * i, cnt - 1)) * C + c) * 2);
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (qb + 256 * i < cnt) t += fn(v[i], qbase + qb + 256 * i);
  }
  return t;
}

// This thread's chunk pairs of up to 2 groups x NI chunks (chunk q0_g + lane + 256 i), all loaded
// up front: the second pass over the partials (and every group) then costs no memory round trip.
// sum(g, fn) accumulates in the same chunk order as cgl_fin_sum.
template <int NI>
struct CglFinCache {
  typedef double f64x2 __attribute__((ext_vector_type(2)));
  f64x2 v[2][NI];
  int cnt, lane;
  __device__ __forceinline__ void load(const double* part, long gstride, int groups, int cnt_, int C, int c,
                                       int lane_, long q0 = 0) {
    typedef const CGL_GLOBAL f64x2* gcd2p;
    cnt = cnt_;
    lane = lane_;
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int q = min(lane + 256 * i, cnt - 1);
        const int gg = min(g, groups - 1);
        v[g][i] = *(gcd2p)(part + ((q0 + gg * gstride + q) * C + c) * 2);
      }
  }
  template <class Fn>
  __device__ __forceinline__ double sum(int g, Fn fn, int qbase = 0) const {
    // the group is selected, not indexed: a runtime index into v[][] puts the cache in scratch
    double t = 0.0;
#pragma unroll
    for (int i = 0; i < NI; ++i)
      if (lane + 256 * i < cnt) t += fn(g ? v[1][i] : v[0][i], qbase + lane + 256 * i);
    return t;
  }
};

// channel c's finalize by one workgroup (cgl_bn_finalize; the deferred column-sum finish of
// cgl_conv_wgrad_reduce_multi); red: 4 doubles of LDS
template <class FA>
__device__ __forceinline__ void cgl_bn_finalize_at(const FA& a, int c, double* red) {
  const int lane = threadIdx.x;          // thread index within the channel's workgroup
  const int C = a.C;
  const double* part = a.part;
  // <= 1024 chunks per call and <= 2 calls: every partial this thread needs is loaded once, up front
  CglFinCache<4> fc;
  const bool cached = a.chunks_per_group <= 1024 && a.groups <= 2 && a.mode != 2 && (a.mode == 1 || a.train) &&
                      !a.nocache;
  if (cached) fc.load(part, a.chunks_per_group, a.groups, a.chunks_per_group, C, c, lane);
  auto gsum = [&](int g, auto fn) -> double {
    return cached ? fc.sum(g, fn) : cgl_fin_sum(part, (long)g * a.chunks_per_group, a.chunks_per_group, C, c, lane, fn);
  };
  if (a.mode == 2) {
    const int nch = a.groups * a.chunks_per_group;
    double t = cgl_fin_sum(part, 0, nch, C, c, lane, [](auto v, int) { return (double)v[0]; });
    t = cgl_block_sum_d(t, red);
    if (lane == 0) gst(a.dgamma + c, (float)t);
    return;
  }
  const float w = a.gamma ? gld(a.gamma + c) : 1.f;
  if (a.mode == 1) {
    double dg = 0.0, db = 0.0;
    for (int g = 0; g < a.groups; ++g) {
      double S = gsum(g, [](auto v, int) { return (double)v[0]; });
      double D = gsum(g, [](auto v, int) { return (double)v[1]; });
      S = cgl_block_sum_d(S, red);
      D = cgl_block_sum_d(D, red);
      const float invstd = gld(a.save_invstd + (long)g * C + c);
      const int ng = cgl_fin_rows(a, g);
      if (lane == 0) {
        gst(a.coef0 + (long)g * C + c, (float)(S / ng));
        gst(a.coef1 + (long)g * C + c, (float)D * invstd * invstd / ng);
      }
      dg += D * (double)invstd;
      db += S;
    }
    if (lane == 0) {
      if (a.dgamma) gst(a.dgamma + c, (float)dg);
      if (a.dbeta) gst(a.dbeta + c, (float)db);
    }
    return;
  }
  const float b = a.beta ? gld(a.beta + c) : 0.f;
  if (!a.train) {
    if (lane != 0) return;
    const double invstd = 1.0 / sqrt((double)gld(a.run_var + c) + a.eps);
    const float sc = (float)invstd * w;
    for (int g = 0; g < a.groups; ++g) {
      gst(a.coef0 + (long)g * C + c, sc);
      gst(a.coef1 + (long)g * C + c, b - gld(a.run_mean + c) * sc);
    }
    return;
  }
  float rm = a.run_mean ? gld(a.run_mean + c) : 0.f, rv = a.run_var ? gld(a.run_var + c) : 0.f;
  for (int g = 0; g < a.groups; ++g) {
    double s = gsum(g, [](auto v, int) { return (double)v[0]; });
    s = cgl_block_sum_d(s, red);
    const int ng = cgl_fin_rows(a, g);
    const double n = ng;
    const double mu = s / n;
    const double R = a.R;
    const bool full = ng == a.gr;            // every chunk holds R rows (the common case: one code path)
    double m2 = gsum(g, [&](auto v, int q) {
      const double cnt = full ? R : (double)cgl_fin_chunk_rows(ng, q, a.R);
      if (cnt == 0.0) return 0.0;
      const double dd = v[0] / cnt - mu;
      return (double)v[1] + cnt * dd * dd;
    });
    m2 = cgl_block_sum_d(m2, red);
    const double invstd = 1.0 / sqrt(m2 / n + a.eps);
    const float sc = (float)invstd * w;
    if (lane == 0) {
      gst(a.coef0 + (long)g * C + c, sc);
      gst(a.coef1 + (long)g * C + c, b - (float)mu * sc);
      if (a.save_mean) {
        gst(a.save_mean + (long)g * C + c, (float)mu);
        gst(a.save_invstd + (long)g * C + c, (float)invstd);
      }
    }
    if (a.run_mean) {
      const double mom = a.momentum;
      rm = (float)(mom * mu + (1.0 - mom) * (double)rm);
      rv = (float)(mom * (n > 1 ? m2 / (n - 1) : m2 / n) + (1.0 - mom) * (double)rv);
    }
  }
  if (a.run_mean && lane == 0) {
    gst(a.run_mean + c, rm);
    gst(a.run_var + c, rv);
  }
}

__global__ __launch_bounds__(256) void cgl_bn_finalize(CglBnFinArgs a) {
  __shared__ double red[4];
  cgl_bn_finalize_at(a, (int)blockIdx.x, red);
}


// Sliced training-mode BatchNorm2d finalize for statistics with many chunks (the 32-row chunks a
// conv epilogue writes: 8192 per forward call of the generator's last BatchNorm at B=256): block
// (s, c) merges slice s of channel c's chunks of every call into {mean_s, M2_s} (two passes, fixed
// order), publishes them with agent-scope atomic stores and takes a ticket; the last block of
// channel c merges the S slices in slice order (Chan) and finishes exactly as cgl_bn_finalize mode
// 0.  Tickets are monotonic (the caller zeroes them once; every launch adds S per channel).
#define CGL_FIN_MAXS 64
struct CglBnFinSliced {
  CglBnFinArgs f;
  int S, L;                  // slices per channel, chunks per slice
  double* sl;                // [C][groups][S][2] slice {mean, M2}
  unsigned int* ctr;         // [C] tickets
};

__global__ __launch_bounds__(256) void cgl_bn_finalize_sliced(CglBnFinSliced a) {
  __shared__ double red[4];
  __shared__ double smu[CGL_FIN_MAXS], sm2[CGL_FIN_MAXS];
  __shared__ int last;
  const int s = blockIdx.x, c = blockIdx.y, lane = threadIdx.x;
  const int C = a.f.C, cpg = a.f.chunks_per_group, G = a.f.groups, S = a.S;
  const int q_lo = s * a.L, cnt = min(q_lo + a.L, cpg) - q_lo;
  const double R = a.f.R;
  CglFinCache<2> fc;                     // a slice is <= 512 chunks: <= 2 per thread and call
  if (G <= 2 && a.L <= 512) fc.load(a.f.part, cpg, G, cnt, C, c, lane, q_lo);
  for (int g = 0; g < G; ++g) {
    const long q0 = (long)g * cpg + q_lo;
    auto gsum = [&](auto fn) -> double {
      return (G <= 2 && a.L <= 512) ? fc.sum(g, fn, q_lo) : cgl_fin_sum(a.f.part, q0, cnt, C, c, lane, fn, q_lo);
    };
    const int ng = cgl_fin_rows(a.f, g);
    const bool full = ng == a.f.gr;
    const int srows = full ? cnt * a.f.R : min(max(ng - q_lo * a.f.R, 0), cnt * a.f.R);   // this slice's rows
    double sm = gsum([](auto v, int) { return (double)v[0]; });
    sm = cgl_block_sum_d(sm, red);
    const double mu = full ? sm / (cnt * R) : (srows > 0 ? sm / srows : 0.0);
    double m2 = gsum([&](auto v, int q) {
      const double rq = full ? R : (double)cgl_fin_chunk_rows(ng, q, a.f.R);
      if (rq == 0.0) return 0.0;
      const double dd = v[0] / rq - mu;
      return (double)v[1] + rq * dd * dd;
    });
    m2 = cgl_block_sum_d(m2, red);
    if (lane == 0) {
      double* dst = a.sl + (((long)c * G + g) * S + s) * 2;
      cgl_pubd(dst, mu);
      cgl_pubd(dst + 1, m2);
    }
  }
  if (lane == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // the published words have landed
    const unsigned int old = __hip_atomic_fetch_add((cgl_gu32*)(a.ctr + c), 1u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
    last = (old % (unsigned)S) == (unsigned)(S - 1);
  }
  __syncthreads();
  if (!last) return;
  const float w = a.f.gamma ? gld(a.f.gamma + c) : 1.f;
  const float b = a.f.beta ? gld(a.f.beta + c) : 0.f;
  float rm = a.f.run_mean ? gld(a.f.run_mean + c) : 0.f, rv = a.f.run_var ? gld(a.f.run_var + c) : 0.f;
  for (int g = 0; g < G; ++g) {
    if (lane < S) {
      const double* src = a.sl + (((long)c * G + g) * S + lane) * 2;
      smu[lane] = __longlong_as_double((long long)cgl_ld64(src));
      sm2[lane] = __longlong_as_double((long long)cgl_ld64(src + 1));
    }
    __syncthreads();
    if (lane == 0) {
      const int ng = cgl_fin_rows(a.f, g);
      const bool full = ng == a.f.gr;
      const double n = ng;
      // rows of slice q (all of its chunks' R rows, or the short call's share of them)
      auto qrows = [&](int q) -> double {
        const int rq = (min((q + 1) * a.L, cpg) - q * a.L) * a.f.R;
        return full ? (double)(min((q + 1) * a.L, cpg) - q * a.L) * R : (double)min(max(ng - q * a.L * a.f.R, 0), rq);
      };
      double tot = 0.0;
      for (int q = 0; q < S; ++q) tot += full ? smu[q] * (min((q + 1) * a.L, cpg) - q * a.L) * R : smu[q] * qrows(q);
      const double mu = tot / n;
      double m2 = 0.0;
      for (int q = 0; q < S; ++q) {
        const double dd = smu[q] - mu;
        m2 += sm2[q] + qrows(q) * dd * dd;
      }
      const double invstd = 1.0 / sqrt(m2 / n + a.f.eps);
      const float sc = (float)invstd * w;
      gst(a.f.coef0 + (long)g * C + c, sc);
      gst(a.f.coef1 + (long)g * C + c, b - (float)mu * sc);
      if (a.f.save_mean) {
        gst(a.f.save_mean + (long)g * C + c, (float)mu);
        gst(a.f.save_invstd + (long)g * C + c, (float)invstd);
      }
      if (a.f.run_mean) {
        const double mom = a.f.momentum;
        rm = (float)(mom * mu + (1.0 - mom) * (double)rm);
        rv = (float)(mom * (n > 1 ? m2 / (n - 1) : m2 / n) + (1.0 - mom) * (double)rv);
      }
    }
    __syncthreads();
  }
  if (a.f.run_mean && lane == 0) {
    gst(a.f.run_mean + c, rm);
    gst(a.f.run_var + c, rv);
  }
}

// The discriminator head forward (model/lsgan.py:96-97: out.view(B, -1) -> adv_layer = Linear(C*hw, 1))
// read straight from the NHWC map, with the NCHW view's transpose folded into the loads.  The
// arithmetic is cgl_conv_n1's for this single-tap problem, in its order: lane q owns flat elements
// 4 (q + 64 b) + j, fma-chained over b then j from 0, lanes combined by the same xor tree, then + bias --
// so Y is bitwise what nhwc_to_nchw + dense_fwd(N = 1) produced.  `flat` (may be null) receives the
// NCHW view for adv_layer's weight gradient.
// One row of a one-logit loss (cgl_adv_loss_at's loss 1 / 2 / 3): its loss term l and weight * d(mean loss)/dz (invM = 1 / M)
__device__ __forceinline__ void cgl_adv_row1(float z, int loss, int target, float weight, float invM, float& l,
                                             float& g0) {
  if (loss == 2) {
    const float d = z - (float)target;
    l = d * d;
    g0 = weight * (2.f * d * invM);
  } else {
    const float pr = loss == 3 ? 1.f / (1.f + expf(-z)) : z;
    const float y = (float)target;
    const float lp = fmaxf(logf(pr), -100.f), l1p = fmaxf(logf(1.f - pr), -100.f);
    l = -(y * lp + (1.f - y) * l1p);
    const float gp = weight * invM * (pr - y) / fmaxf((1.f - pr) * pr, 1e-12f);
    g0 = loss == 3 ? gp * (1.f - pr) * pr : gp;
  }
}

// coef: the row's BatchNorm applied to every loaded value (v = fmaf(x, coef[cg + c], coef[shb + cg + c]), the
// cgl_eltwise mode-0 arithmetic, act none: the head of the D step / G-loss pass reads the PRE-BatchNorm map)
__device__ __forceinline__ float cgl_dense1_row(const float* __restrict__ X, const float* __restrict__ W,
                                                float* __restrict__ flat, int row, int q, int C, int hw,
                                                const float* __restrict__ coef = nullptr, int cg = 0, int shb = 0) {
  const int per = C * hw, nb = per >> 8;     // per % 256 == 0, nb <= 4
  const float* __restrict__ x = X + (long)row * per;
  f32x4 v[4], w[4];
#pragma unroll
  for (int bb = 0; bb < 4; ++bb) {
    if (bb < nb) {
      const int k0 = 4 * (q + 64 * bb);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = (k0 + j) / hw, s = k0 + j - c * hw;
        v[bb][j] = gld(x + s * C + c);
        if (coef) v[bb][j] = fmaf(v[bb][j], gld(coef + cg + c), gld(coef + shb + cg + c));
      }
      w[bb] = *(gcf4p)(W + k0);
    }
  }
  float acc = 0.f;
#pragma unroll
  for (int bb = 0; bb < 4; ++bb)
    if (bb < nb) {
      acc = fmaf(v[bb][0], w[bb][0], acc);
      acc = fmaf(v[bb][1], w[bb][1], acc);
      acc = fmaf(v[bb][2], w[bb][2], acc);
      acc = fmaf(v[bb][3], w[bb][3], acc);
    }
  for (int o = 1; o < 64; o <<= 1) acc += __shfl_xor(acc, o);
  if (flat) {
#pragma unroll
    for (int bb = 0; bb < 4; ++bb)
      if (bb < nb) *(gf4p)(flat + (long)row * per + 4 * (q + 64 * bb)) = v[bb];
  }
  return acc;
}

__global__ __launch_bounds__(256) void cgl_dense1_fwd_nhwc_k(const float* __restrict__ X, const float* __restrict__ W,
                                                             const float* __restrict__ b, float* __restrict__ Y,
                                                             float* __restrict__ flat, int n, int C, int hw) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), q = threadIdx.x & 63;
  if (row >= n) return;                      // wave-uniform
  const float acc = cgl_dense1_row(X, W, flat, row, q, C, hw);
  if (q == 0) gst(Y + row, acc + (b ? gld(b) : 0.f));
}

// The discriminator head of model/lsgan.py as ONE launch: adv_layer's forward from the NHWC map
// (cgl_dense1_fwd_nhwc's arithmetic; `flat` as there), each row's adversarial-loss term and gradient
// (cgl_adv_loss_at's arithmetic, cgl_adv_row1) and the row's input gradient into the NHWC map
// (cgl_dense1_bwd_nhwc_k's products) -- everything of a row depends on that row alone, so the three launches
// (forward, loss head(s), input gradient) become one.  The calls (the D step's real and fake halves, or the
// G-loss pass's one call) each keep their own target, weight and batch mean; a short first call (nv) gives its
// padding rows no loss and a zero gradient.  The batch-mean losses: every wave publishes its row's loss term
// (agent-scope atomic store), the workgroup takes a monotonic ticket, and the last workgroup to arrive sums
// the terms in cgl_adv_loss_at's order (thread t: rows t, t + 256, ... in double; then the 256 partials in
// order), so every output is bitwise what the three separate launches give.
struct CglHeadCall {
  int n0, n, target;
  float weight;
  float* loss_out;
  const int* nv;
};
struct CglDHeadArgs {
  const float* X; const float* W; const float* b;
  float* Y; float* flat; float* dY; float* dX;
  int n, C, hw, loss, ncalls;
  CglHeadCall call[2];
  float* lrow;               // [n] published loss terms
  unsigned int* ticket;      // monotonic (zeroed once by the caller)
  const float* coef; int groups;   // X's BatchNorm [2][groups][C] applied in the loads (cgl_dense1_row), or null
};
__global__ __launch_bounds__(256) void cgl_dense1_head_k(CglDHeadArgs a) {
  __shared__ double s_acc[256];
  __shared__ int s_last;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), q = threadIdx.x & 63;
  if (row < a.n) {                           // wave-uniform
    const int bg = a.coef ? min(row / (a.n / a.groups), a.groups - 1) : 0;
    const float acc = cgl_dense1_row(a.X, a.W, a.flat, row, q, a.C, a.hw, a.coef, bg * a.C, a.groups * a.C);
    const float z = acc + (a.b ? gld(a.b) : 0.f);
    const int ci = (a.ncalls > 1 && row >= a.call[1].n0) ? 1 : 0;
    const int n0 = ci ? a.call[1].n0 : a.call[0].n0, nc = ci ? a.call[1].n : a.call[0].n;
    const int* nvp = ci ? a.call[1].nv : a.call[0].nv;
    const int M = nvp ? min(max(gldi(nvp), 1), nc) : nc;
    const float invM = 1.f / (float)M;
    float l = 0.f, g = 0.f;
    if (row - n0 < M)
      cgl_adv_row1(z, a.loss, ci ? a.call[1].target : a.call[0].target, ci ? a.call[1].weight : a.call[0].weight,
                   invM, l, g);
    if (q == 0) {
      gst(a.Y + row, z);
      gst(a.dY + row, g);
      __hip_atomic_store((cgl_gu32*)(a.lrow + row), __float_as_uint(l), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // input gradient, NHWC: dX[row][s][c] = g * W[c * hw + s] (float4 per lane, cgl_dense1_bwd_nhwc_k's products)
    const int per = a.C * a.hw, nb = per >> 8;
#pragma unroll
    for (int bb = 0; bb < 4; ++bb)
      if (bb < nb) {
        const int e = 4 * (q + 64 * bb);
        const int sp = e / a.C, c = e - sp * a.C;
        f32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = g * gld(a.W + (long)(c + j) * a.hw + sp);
        *(gf4p)(a.dX + (long)row * per + e) = o;
      }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave's published term has landed
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned int old = __hip_atomic_fetch_add((cgl_gu32*)a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (old % gridDim.x) == gridDim.x - 1;
  }
  __syncthreads();
  if (!s_last) return;
  for (int ci = 0; ci < a.ncalls; ++ci) {
    const int n0 = ci ? a.call[1].n0 : a.call[0].n0, nc = ci ? a.call[1].n : a.call[0].n;
    const int* nvp = ci ? a.call[1].nv : a.call[0].nv;
    const int M = nvp ? min(max(gldi(nvp), 1), nc) : nc;
    double acc = 0.0;
    for (int r = threadIdx.x; r < M; r += 256)
      acc += (double)__uint_as_float(
          __hip_atomic_load((cgl_gu32*)(a.lrow + n0 + r), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    s_acc[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
      double t = 0.0;
      for (int k = 0; k < 256; ++k) t += s_acc[k];
      float* lo = ci ? a.call[1].loss_out : a.call[0].loss_out;
      if (lo) gst(lo, (float)(t / M));
    }
    __syncthreads();
  }
}

// Weight + bias gradient of a one-output Linear (the discriminator's adv_layer, model/lsgan.py:90-97, on the
// NCHW-flattened map): dW[k] = sum_m dY[m] X[m][k], db = sum_m dY[m] in ONE launch (the implicit-GEMM weight
// gradient took four: partial tiles, their reduce, the bias column sum and its finalize, for 0.27 MFLOP).
// Block b < gridDim.x - 1: 16 columns x 16 row lanes (a wave reads 4 rows x 64 contiguous bytes); lane l sums
// rows l, l + 16, ... in order in double (exact products), 32 loads in flight (M <= 512: one batch); the 16 lanes
// are added in lane order.  The last block: db, thread t summing rows t, t + 256, ... then the 256 partials in order.
// block bid of nblk (cgl_dense1_wgrad_k; the deferred reductions' launch, cgl_conv_wgrad_reduce_multi)
__device__ __forceinline__ void cgl_dense1_wgrad_at(const float* __restrict__ dY, const float* __restrict__ X,
                                                    float* __restrict__ dW, float* __restrict__ db, int M, int K,
                                                    int bid, int nblk, double* red) {
  const int t = threadIdx.x;
  if (bid == nblk - 1) {      // the bias block (uniform)
    double acc = 0.0;
    for (int m = t; m < M; m += 256) acc += (double)gld(dY + m);
    red[t] = acc;
    __syncthreads();
    if (t == 0) {
      double s = 0.0;
      for (int i = 0; i < 256; ++i) s += red[i];
      if (db) gst(db, (float)s);
    }
    return;
  }
  const int kl = t & 15, ml = t >> 4;
  const int k = bid * 16 + kl, kc = min(k, K - 1);
  double acc = 0.0;
  for (int m0 = ml; m0 < M; m0 += 16 * 32) {
    float xv[32], dv[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const int m = min(m0 + 16 * i, M - 1);
      xv[i] = gld(X + (long)m * K + kc);
      dv[i] = gld(dY + m);
    }
#pragma unroll
    for (int i = 0; i < 32; ++i)
      if (m0 + 16 * i < M) acc += (double)dv[i] * (double)xv[i];
  }
  red[t] = acc;
  __syncthreads();
  if (ml == 0 && k < K) {
    double s = 0.0;
    for (int l = 0; l < 16; ++l) s += red[16 * l + kl];
    gst(dW + k, (float)s);
  }
}

__global__ __launch_bounds__(256) void cgl_dense1_wgrad_k(const float* __restrict__ dY, const float* __restrict__ X,
                                                          float* __restrict__ dW, float* __restrict__ db, int M,
                                                          int K) {
  __shared__ double red[256];
  cgl_dense1_wgrad_at(dY, X, dW, db, M, K, (int)blockIdx.x, (int)gridDim.x, red);
}

// The deferred split reductions of several weight gradients (cgl_conv_wgrad_defer_begin / _end) and the
// single-input-channel kernel's finish (cgl_conv_c1_wgrad_fin) as ONE launch: block ranges [begin[q],
// begin[q + 1]) run reduction q, blocks from begin[n] the c1 finish, then the column-sum finishes, then the
// one-output dense weight gradient.  Each block computes exactly what it
// computes in its own launch (same function, same block index), so the gradients are bitwise unchanged.
#define CGL_WDEFER_MAX 4
#define CGL_WDEFER_FIN 3
struct CglWgradReduceMulti {
  int n, c1_blocks, nfin;
  int begin[CGL_WDEFER_MAX + 1];
  int fbeg[CGL_WDEFER_FIN + 1];   // block offsets of the column-sum finishes, from begin[n] + c1_blocks
  CglWgradReduceArgs r[CGL_WDEFER_MAX];
  CglC1Args c1;
  CglBnFinArgs fin[CGL_WDEFER_FIN];   // deferred column-sum finishes (bias gradients: cgl_colsum_finalize, col_sum)
  // a deferred one-output dense weight gradient (cgl_dense1_wgrad_k: the D head's adv_layer), d1_blocks > 0
  const float* d1_dy; const float* d1_x; float* d1_dw; float* d1_db; int d1_M, d1_K, d1_blocks;
  // the round's device counters (cgl_conv_wgrad_defer_counters), one extra last block when cnt != null:
  // *cnt_snap = cnt[cnt_si], then cnt[0 .. cnt_n) += cnt_v (nothing else in the launch reads them)
  int* cnt; int* cnt_snap; int cnt_n, cnt_v, cnt_si;
};

__global__ __launch_bounds__(256) void cgl_conv_wgrad_reduce_multi(CglWgradReduceMulti m) {
  __shared__ double red[256];
  const int b = blockIdx.x, n = m.n;
  const int fend = m.begin[n] + m.c1_blocks + m.fbeg[m.nfin];
  if (b >= fend + m.d1_blocks) {     // the counters block
    const int t = threadIdx.x;
    const int snap = m.cnt[m.cnt_si];
    __syncthreads();                 // (every lane has read the snapshot value before lane 0..n-1 add)
    if (t == 0) *m.cnt_snap = snap;
    if (t < m.cnt_n) m.cnt[t] += m.cnt_v;
    return;
  }
  if (b >= fend) {
    cgl_dense1_wgrad_at(m.d1_dy, m.d1_x, m.d1_dw, m.d1_db, m.d1_M, m.d1_K, b - fend, m.d1_blocks, red);
    return;
  }
  if (b >= m.begin[n] + m.c1_blocks) {
    const int f = b - m.begin[n] - m.c1_blocks;
    if (m.nfin > 2 && f >= m.fbeg[2]) cgl_bn_finalize_at(m.fin[2], f - m.fbeg[2], red);
    else if (m.nfin > 1 && f >= m.fbeg[1]) cgl_bn_finalize_at(m.fin[1], f - m.fbeg[1], red);
    else cgl_bn_finalize_at(m.fin[0], f, red);
    return;
  }
  if (b >= m.begin[n]) {
    cgl_conv_c1_wgrad_fin_at(m.c1, b - m.begin[n], red);
    return;
  }
  // (constant member indices: a runtime index into the by-value argument would copy it to scratch)
  if (n > 3 && b >= m.begin[3]) cgl_conv_wgrad_reduce_at(m.r[3], b - m.begin[3], red);
  else if (n > 2 && b >= m.begin[2]) cgl_conv_wgrad_reduce_at(m.r[2], b - m.begin[2], red);
  else if (n > 1 && b >= m.begin[1]) cgl_conv_wgrad_reduce_at(m.r[1], b - m.begin[1], red);
  else cgl_conv_wgrad_reduce_at(m.r[0], b, red);
}

// Elementwise NHWC passes (float4 over channels; C % 4 == 0):
//   mode 0  Y = act(X * coef0[g][c] + coef1[g][c])                               (BatchNorm2d apply)
//   mode 1  dX = (g - coef0[g][c] - (X - mean[g][c]) coef1[g][c]) invstd[g][c] gamma[c],
//           g = dY * leaky'(post)  (BatchNorm2d backward apply), then * drop * leaky'(post_out)
//   mode 2  dX = dY * leaky'(post_out) * drop                      (Dropout2d + LeakyReLU backward)
//   mode 3  dX = dY * (1 - Y^2)                                                  (Tanh backward)
struct CglEltArgs {
  int mode, rows, C, gr, hw, act;
  int row0;                  // the first row of X / out is row row0 of the whole tensor (its BatchNorm group)
  float slope;
  const float* X; const float* dY; const float* post;
  const float* coef0; const float* coef1; const float* mean; const float* invstd; const float* gamma;
  const float* post_out; const float* drop;
  float* out;
  const int* nv;             // mode 1, short first call: rows >= *nv * hw of group 0 are padding -> dX = 0
  const float* psc; int psc_ld;   // mode 1: LeakyReLU'(post) from the forward's scale / shift (CglChanArgs)
  // cgl_eltwise1, C == 1, one element per thread: also the column-sum partials of the output per 256-row chunk
  // (= block), {sum, 0} -- bitwise cgl_chan_reduce mode 2 with R = 256 over the stored output
  double* colsum;
};

// one float4 of cgl_eltwise mode 1 (the BatchNorm2d backward apply) at element e = (row r, channel c), BatchNorm
// group g (gc = g C + c), nvr: the data rows of a short first call (cgl_eltwise, cgl_bnb_apply_colsum)
__device__ __forceinline__ f32x4 cgl_elt_bnb4(const CglEltArgs& a, long e, int r, int c, int g, long gc, int nvr) {
  const float sl = a.slope;
  f32x4 o;
  const f32x4 x = *(gcf4p)(a.X + e), dy = *(gcf4p)(a.dY + e);
  const f32x4 gm = *(gcf4p)(a.coef0 + gc), kk = *(gcf4p)(a.coef1 + gc);
  const f32x4 mu = *(gcf4p)(a.mean + gc), is = *(gcf4p)(a.invstd + gc), w = *(gcf4p)(a.gamma + c);
  f32x4 p = dy;
  if (a.psc) {
    const f32x4 ps = *(gcf4p)(a.psc + c), ph = *(gcf4p)(a.psc + a.psc_ld + c);
#pragma unroll
    for (int j = 0; j < 4; ++j) p[j] = fmaf(x[j], ps[j], ph[j]);
  } else if (a.post) {
    p = *(gcf4p)(a.post + e);
  }
  const bool pon = a.psc || a.post;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float gg = pon ? (p[j] > 0.f ? dy[j] : dy[j] * sl) : dy[j];
    o[j] = (gg - gm[j] - (x[j] - mu[j]) * kk[j]) * is[j] * w[j];
  }
  if (a.post_out) {
    const f32x4 po = *(gcf4p)(a.post_out + e);
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = po[j] > 0.f ? o[j] : o[j] * sl;
  }
  if (a.drop) {
    const f32x4 dm = *(gcf4p)(a.drop + (long)(r / a.hw) * a.C + c);
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] *= dm[j];
  }
  if (g == 0 && r + a.row0 >= nvr) o = f32x4{0.f, 0.f, 0.f, 0.f};   // padding of a short first call
  return o;
}

// cgl_eltwise mode 1 (the BatchNorm2d backward apply) over 256-row chunks, one per workgroup, that also writes the
// per-chunk column sums of its output in cgl_chan_reduce4 mode 2's lane mapping, order and layout (R = 256:
// part[chunk][c] = {sum, 0}) -- bitwise the apply followed by col_sum's channel reduction over the stored output
// (the bias gradient of the conv whose output gradient this is), one pass over the tensor fewer.  Rows of a lane
// in batches of NB (their loads in flight together), accumulated in row order.
#ifndef CGL_BNB_NB
#define CGL_BNB_NB 4   // rows of a lane in flight together (16 measured the same, gpurun_out/r06zg)
#endif
template <int NB>
__global__ __launch_bounds__(256) void cgl_bnb_apply_colsum(CglEltArgs a, double* __restrict__ part) {
  __shared__ double s0[1024];
  const int C = a.C, CW = C >> 2, rp = 256 / CW;
  const int cs = threadIdx.x % CW, rl = threadIdx.x / CW, c = 4 * cs;
  const int r0 = blockIdx.x * 256, r1 = min(r0 + 256, a.rows);
  const int nvr = cgl_nv_rows(a.nv, a.hw, a.gr);
  double x0[4] = {0.0, 0.0, 0.0, 0.0};
  for (int rb = r0 + rl; rb < r1; rb += NB * rp) {
    f32x4 o[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int r = min(rb + i * rp, r1 - 1);
      const int g = (r + a.row0) / a.gr;
      o[i] = cgl_elt_bnb4(a, (long)r * C + c, r, c, g, (long)g * C + c, nvr);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i)
      if (rb + i * rp < r1) {
        *(gf4p)(a.out + (long)(rb + i * rp) * C + c) = o[i];
#pragma unroll
        for (int j = 0; j < 4; ++j) x0[j] += (double)o[i][j];
      }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) s0[threadIdx.x * 4 + j] = x0[j];
  __syncthreads();
  if (rl == 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      double t0 = 0.0, t1 = 0.0;
      for (int q = 0; q < rp; ++q) t0 += s0[(q * CW + cs) * 4 + j];
      part[((long)blockIdx.x * C + c + j) * 2] = t0;
      part[((long)blockIdx.x * C + c + j) * 2 + 1] = t1;
    }
  }
}

__global__ __launch_bounds__(256) void cgl_eltwise(CglEltArgs a) {
  const long n4 = (long)a.rows * a.C / 4;
  const int C = a.C;
  const float sl = a.slope;
  const int nvr = a.mode == 1 ? cgl_nv_rows(a.nv, a.hw, a.gr) : a.gr;
  // 32-bit index arithmetic when the tensor allows it (a 64-bit division per float4 costs more VALU
  // than the element work)
  const bool small = n4 < (1L << 29);
  for (long q = (long)blockIdx.x * 256 + threadIdx.x; q < n4; q += (long)gridDim.x * 256) {
    const long e = q * 4;
    int r, c;
    if (small) {
      const unsigned eu = (unsigned)e, ru = eu / (unsigned)C;
      r = (int)ru;
      c = (int)(eu - ru * (unsigned)C);
    } else {
      r = (int)(e / C);
      c = (int)(e - (long)r * C);
    }
    const int g = (r + a.row0) / a.gr;
    const long gc = (long)g * C + c;
    f32x4 o;
    if (a.mode == 0) {
      const f32x4 x = *(gcf4p)(a.X + e);
      const f32x4 s = *(gcf4p)(a.coef0 + gc), h = *(gcf4p)(a.coef1 + gc);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v = fmaf(x[j], s[j], h[j]);
        if (a.act == CGL_EPI_ACT_LEAKY) v = v > 0.f ? v : v * sl;
        o[j] = v;
      }
    } else if (a.mode == 1) {
      o = cgl_elt_bnb4(a, e, r, c, g, gc, nvr);
    } else if (a.mode == 2) {
      const f32x4 dy = *(gcf4p)(a.dY + e);
      o = dy;
      if (a.post_out) {
        const f32x4 po = *(gcf4p)(a.post_out + e);
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = po[j] > 0.f ? o[j] : o[j] * sl;
      }
      if (a.drop) {
        const f32x4 dm = *(gcf4p)(a.drop + (long)(r / a.hw) * C + c);
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] *= dm[j];
      }
    } else {
      const f32x4 dy = *(gcf4p)(a.dY + e), y = *(gcf4p)(a.X + e);
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = cgl_dtanh(dy[j], y[j]);
    }
    *(gf4p)(a.out + e) = o;
  }
}

// Input gradient of a one-output Linear over a flattened NCHW feature map (the discriminator head,
// model/lsgan.py:96-97: out.view(B, -1) -> adv_layer), written straight into the NHWC layout of the
// map: dX[m][s][c] = dY[m] * W[c * hw + s].  One product per element (what the K = 1 GEMM computes),
// with the view's transpose folded into the store -- one launch instead of a GEMM and a transpose.
__global__ __launch_bounds__(256) void cgl_dense1_bwd_nhwc_k(const float* __restrict__ dY,
                                                             const float* __restrict__ W, float* __restrict__ dX,
                                                             int n, int C, int hw) {
  const int per = C * hw, q4 = per >> 2;      // C % 4 == 0: a float4 never crosses a pixel
  const int total = n * q4;
  for (int q = blockIdx.x * 256 + threadIdx.x; q < total; q += gridDim.x * 256) {
    const int m = q / q4, e = (q - m * q4) * 4;
    const int s = e / C, c = e - s * C;
    const float d = gld(dY + m);
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = d * gld(W + (long)(c + j) * hw + s);
    *(gf4p)(dX + (long)m * per + e) = o;
  }
}

// Scalar fallback of mode 2 / 3 for C % 4 != 0 (single-channel tensors: the generator image).
__global__ __launch_bounds__(256) void cgl_eltwise1(CglEltArgs a) {
  const long n = (long)a.rows * a.C;
  float ov = 0.f;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const int r = (int)(e / a.C), c = (int)(e - (long)r * a.C);
    float o = gld(a.dY + e);
    if (a.mode == 3) {
      const float y = gld(a.X + e);
      o = cgl_dtanh(o, y);
    } else {
      if (a.post_out) o = gld(a.post_out + e) > 0.f ? o : o * a.slope;
      if (a.drop) o *= gld(a.drop + (long)(r / a.hw) * a.C + c);
    }
    gst(a.out + e, o);
    ov = o;
  }
  if (a.colsum) {      // (uniform) the chunk's rows summed in row order, as cgl_chan_reduce's thread 0 does
    __shared__ double s0[256];
    const long e = (long)blockIdx.x * 256 + threadIdx.x;
    s0[threadIdx.x] = e < n ? (double)ov : 0.0;
    __syncthreads();
    if (threadIdx.x == 0) {
      double t = 0.0;
      for (int q = 0; q < 256; ++q) t += s0[q];
      a.colsum[(long)blockIdx.x * 2] = t;
      a.colsum[(long)blockIdx.x * 2 + 1] = 0.0;
    }
  }
}

// Dropout2d(p) scale per (image, channel): 1/(1-p) with probability 1-p, else 0 (torch:
// bernoulli_(1 - p) then div_(1 - p)).  Philox4x32-10 keyed by seed, counter = (index, ctr).
__global__ __launch_bounds__(256) void cgl_dropout_mask_k(float* mask, long n, float keep, float scale,
                                                          unsigned long long seed, unsigned long long ctr) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint32_t c[4] = {(uint32_t)i, (uint32_t)(i >> 32), (uint32_t)ctr, (uint32_t)(ctr >> 32) ^ 0x5bd1e995u};
  cgl_philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const float u = (float)(c[0] >> 8) * (1.0f / 16777216.0f);   // [0, 1), 24 bits
  gst(mask + i, u < keep ? scale : 0.f);
}

// Several Dropout2d masks (every mask of a round: one launch instead of one per layer and call);
// mask j is exactly cgl_dropout_mask_k(mask[j], n[j], keep, scale, seed, ctr[j]).
#define CGL_MASKS_MAX 16
struct CglMasksArgs {
  int nm;
  float keep, scale;
  unsigned long long seed;
  float* mask[CGL_MASKS_MAX];
  long n[CGL_MASKS_MAX];
  unsigned long long ctr[CGL_MASKS_MAX];
  int blk_begin[CGL_MASKS_MAX];
  const int* rdev;                  // optional device round: counter j = ctr[j] + rstride * (*rdev)
  unsigned long long rstride;
};

__device__ __forceinline__ void cgl_dropout_masks_at(const CGL_AS4 CglMasksArgs* A, int b) {
  int q = 0;
  for (int j = 1; j < A->nm; ++j)
    if (b >= A->blk_begin[j]) q = j;
  const long i = (long)(b - A->blk_begin[q]) * 256 + threadIdx.x;
  if (i >= A->n[q]) return;
  const unsigned long long ctr = A->ctr[q] + (A->rdev ? A->rstride * (unsigned long long)gldi(A->rdev) : 0ull),
                           seed = A->seed;
  uint32_t c[4] = {(uint32_t)i, (uint32_t)(i >> 32), (uint32_t)ctr, (uint32_t)(ctr >> 32) ^ 0x5bd1e995u};
  cgl_philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const float u = (float)(c[0] >> 8) * (1.0f / 16777216.0f);
  gst(A->mask[q] + i, u < A->keep ? A->scale : 0.f);
}

__global__ __launch_bounds__(256) void cgl_dropout_masks_k(CglMasksArgs) {
  typedef const CGL_AS4 CglMasksArgs* KA;
  cgl_dropout_masks_at((KA)__builtin_amdgcn_kernarg_segment_ptr(), blockIdx.x);
}

// NCHW <-> NHWC for one batch: X [n][c][hw] -> Y [n][hw][c] (to_nhwc) or back.  32x32 tiles in LDS.
__global__ __launch_bounds__(256) void cgl_transpose_k(const float* X, float* Y, int rows, int cols) {
  // per image: X [rows][cols] -> Y [cols][rows]
  __shared__ float t[32][33];
  const long base = (long)blockIdx.z * rows * cols;
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int k = ty; k < 32; k += 8) {
    const int r = r0 + k, c = c0 + tx;
    if (r < rows && c < cols) t[k][tx] = gld(X + base + (long)r * cols + c);
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int c = c0 + k, r = r0 + tx;
    if (r < rows && c < cols) gst(Y + base + (long)c * rows + r, t[tx][k]);
  }
}

// Adversarial loss of one forward call (mean over M rows) and its gradient, one workgroup,
// fixed-order double reduction:
//   0 CE2:  nn.CrossEntropyLoss on 2 logits (capgan.py:311)
//   1 BCE:  nn.BCELoss on probabilities, log clamped at -100 (CGLGAN/2DMG/main.py:336)
//   2 MSE:  nn.MSELoss (LSGAN objective for the model/lsgan.py discriminator; parity vs torch)
//   3 BCE on logits through nn.Sigmoid (Sigmoid + BCELoss, for the model/lsgan.py logit)
// grad = weight * d(mean loss)/dx, written when non-null.
// nv (may be null): only the first *nv rows are a batch (DataLoader's short final batch): the mean runs
// over them and the other rows get a zero gradient.
__device__ __forceinline__ void cgl_adv_loss_at(const float* x, int Mall, int C, int loss, int target, float weight,
                                                float* loss_out, float* grad, const int* nv) {
  __shared__ double s[256];
  double acc = 0.0;
  const int M = nv ? min(max(gldi(nv), 1), Mall) : Mall;
  const float invM = 1.f / (float)M;
  if (grad && M < Mall)
    for (int r = M + threadIdx.x; r < Mall; r += 256) {
      if (loss == 0) {
        gst(grad + 2 * r, 0.f);
        gst(grad + 2 * r + 1, 0.f);
      } else {
        gst(grad + r, 0.f);
      }
    }
  for (int r = threadIdx.x; r < M; r += 256) {
    float l, g0 = 0.f, g1 = 0.f;
    if (loss == 0) {
      const float z0 = gld(x + 2 * r), z1 = gld(x + 2 * r + 1);
      const float mx = fmaxf(z0, z1);
      const float lse = logf(expf(z0 - mx) + expf(z1 - mx));
      const float o0 = z0 - mx - lse, o1 = z1 - mx - lse;
      l = -(target == 0 ? o0 : o1);
      const float w = weight * invM;
      g0 = (target == 0 ? -w : 0.f) + expf(o0) * w;
      g1 = (target == 1 ? -w : 0.f) + expf(o1) * w;
    } else {
      cgl_adv_row1(gld(x + r), loss, target, weight, invM, l, g0);
    }
    acc += (double)l;
    if (grad) {
      if (loss == 0) {
        gst(grad + 2 * r, g0);
        gst(grad + 2 * r + 1, g1);
      } else {
        gst(grad + r, g0);
      }
    }
  }
  s[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int q = 0; q < 256; ++q) t += s[q];
    if (loss_out) gst(loss_out, (float)(t / M));
  }
}
__global__ __launch_bounds__(256) void cgl_adv_loss_k(const float* x, int Mall, int C, int loss, int target,
                                                      float weight, float* loss_out, float* grad, const int* nv) {
  cgl_adv_loss_at(x, Mall, C, loss, target, weight, loss_out, grad, nv);
}

// Multi-tensor Adam (torch 2.10 _single_tensor_adam op order, see cgl_adam in cgl_kernels.hip);
// bias corrections are launch arguments, so no upload and no host sync.
#define CGL_ADAM_MAXT 32
struct CglAdamMulti {
  int nt;
  float* p[CGL_ADAM_MAXT];
  const float* g[CGL_ADAM_MAXT];
  float* m[CGL_ADAM_MAXT];
  float* v[CGL_ADAM_MAXT];
  long n[CGL_ADAM_MAXT];
  int blk[CGL_ADAM_MAXT + 1];
  float step_size, bc2sqrt, b2, w1, w2, eps;
  const int* step_dev;      // optional: completed steps on the device; this update is step *step_dev + 1
  double lr, beta1, beta2;  //   (its bias corrections computed here as cgl_adam_multi does on the host)
};

__global__ __launch_bounds__(256) void cgl_adam_multi_k(CglAdamMulti a) {
  __shared__ float s_sc[2];
  float step_size = a.step_size, bc2sqrt = a.bc2sqrt;
  if (a.step_dev) {
    if (threadIdx.x == 0) {
      const double st = (double)(gldi(a.step_dev) + 1);
      s_sc[0] = (float)(a.lr / (1.0 - pow(a.beta1, st)));
      s_sc[1] = (float)pow(1.0 - pow(a.beta2, st), 0.5);
    }
    __syncthreads();
    step_size = s_sc[0];
    bc2sqrt = s_sc[1];
  }
  const int b = blockIdx.x;
  int t = 0;
  for (int q = 1; q < a.nt; ++q)
    if (b >= a.blk[q]) t = q;
  const long i = (long)(b - a.blk[t]) * 256 + threadIdx.x;
  if (i >= a.n[t]) return;
  float* p = a.p[t];
  float* m = a.m[t];
  float* v = a.v[t];
  const float g = gld(a.g[t] + i);
  const float mm = cgl_lerp(gld(m + i), g, a.w1);
  const float vv = __fadd_rn(__fmul_rn(gld(v + i), a.b2), __fmul_rn(__fmul_rn(a.w2, g), g));
  gst(m + i, mm);
  gst(v + i, vv);
  const float denom = sqrtf(vv) / bc2sqrt + a.eps;
  gst(p + i, gld(p + i) + (-step_size) * mm / denom);
}

// ------------------------------------------------------------------------------------------
// Device-side round state of the fused conv round (ConvGanStep(graph=True)): every per-round value
// the eager round passes from the host -- the z stream's round, the Dropout2d counters, the Adam
// steps, the sampler position -- is read from a small device counter block instead, so one captured
// round replays as a hipGraph; the round's last launch advances the counters.
__global__ __launch_bounds__(256) void cgl_normal_dev_k(float* out, long n, unsigned long long seed, const int* round,
                                                        int stream_id) {
  cgl_normal_at((long)blockIdx.x * 256 + threadIdx.x, out, n, seed, (uint32_t)gldi(round), stream_id);
}

// real batch of round R (DataLoader(shuffle=True), capgan.py:282,326-331): each pass over the n_src rows is
// a keyed Feistel permutation of [0, n_src) (the MLP prologue's sampler) cut into ceil(n_src / nrows)
// batches, the last one short (n_src mod nrows rows); round R takes batch R of the stream.  nv_out (may be
// null) receives the batch's real rows; rows past a short batch copy a valid dummy row (the consumers
// leave them out: cgl_nv_rows).  With nv_out null the pass is cut drop_last (whole batches only).  One
// workgroup per row, float4 copies.
__device__ __forceinline__ void cgl_sample_rows_at(const float* src, int n_src, int nrows, int rowf,
                                                   unsigned long long seed, const int* round, float* dst, int* nv_out,
                                                   int r) {
  uint32_t ep, j;
  if (nv_out) {
    const long nb = (n_src + nrows - 1) / nrows;
    const long bpos = gldi(round);
    ep = (uint32_t)(bpos / nb);
    const long b = bpos % nb;
    const long jj = b * nrows + r;
    j = (uint32_t)(jj < n_src ? jj : n_src - 1);
    if (r == 0 && threadIdx.x == 0) nv_out[0] = (int)(n_src - b * nrows < nrows ? n_src - b * nrows : nrows);
  } else {
    const long per = (long)(n_src / nrows) * nrows;
    const long pos = (long)gldi(round) * nrows + r;
    ep = (uint32_t)(pos / per);
    j = (uint32_t)(pos % per);
  }
  const uint32_t idx = cgl_permute(j, (uint32_t)n_src, (uint32_t)seed ^ (ep * 0x85ebca6bu + 0x1234567u));
  const f32x4* s4 = (const f32x4*)(src + (long)idx * rowf);
  f32x4* d4 = (f32x4*)(dst + (long)r * rowf);
  for (int c = threadIdx.x; c < rowf / 4; c += 256) *(gf4p)(d4 + c) = *(gcf4p)(s4 + c);
}

__global__ __launch_bounds__(256) void cgl_sample_rows_k(const float* src, int n_src, int nrows, int rowf,
                                                         unsigned long long seed, const int* round, float* dst,
                                                         int* nv_out) {
  cgl_sample_rows_at(src, n_src, nrows, rowf, seed, round, dst, nv_out, blockIdx.x);
}

// The conv round's independent start-of-round launches as ONE launch (cgl_conv_batch_begin / _end): the weight
// packing, the Dropout2d masks, the z draw and the real-batch sampler read and write disjoint buffers, so their
// blocks can share a grid: [pack | masks | normal | sample] by block range, each block running its kernel's body.
struct CglAdvArgs {
  const float* x; int Mall, C, loss, target; float weight; float* loss_out; float* grad; const int* nv;
};
struct CglConvBeginArgs {
  CglPackMultiArgs pack;
  CglMasksArgs masks;
  CglAdvArgs adv[2];                  // up to two adversarial-loss heads (one block each: the D step's two calls)
  int pb, mb, nb, sb, lb;             // block counts of the parts (0: absent)
  float* n_out; long n_n; unsigned long long n_seed; const int* n_round; int n_sid;
  const float* s_src; int s_nsrc, s_nrows, s_rowf; unsigned long long s_seed; const int* s_round; float* s_dst;
  int* s_nv;
};
static_assert(sizeof(CglConvBeginArgs) <= 4096, "the batched launch's arguments must fit the kernarg segment");
__global__ __launch_bounds__(256) void cgl_conv_begin_k(CglConvBeginArgs) {
  typedef const CGL_AS4 CglConvBeginArgs* KA;
  const KA A = (KA)__builtin_amdgcn_kernarg_segment_ptr();
  int b = blockIdx.x;
  if (b < A->pb) { cgl_conv_pack_at(&A->pack, b); return; }
  b -= A->pb;
  if (b < A->mb) { cgl_dropout_masks_at(&A->masks, b); return; }
  b -= A->mb;
  if (b < A->nb) {
    cgl_normal_at((long)b * 256 + threadIdx.x, A->n_out, A->n_n, A->n_seed, (uint32_t)gldi(A->n_round), A->n_sid);
    return;
  }
  b -= A->nb;
  if (b < A->sb) {
    cgl_sample_rows_at(A->s_src, A->s_nsrc, A->s_nrows, A->s_rowf, A->s_seed, A->s_round, A->s_dst, A->s_nv, b);
    return;
  }
  b -= A->sb;
  const CGL_AS4 CglAdvArgs* q = &A->adv[b];
  cgl_adv_loss_at(q->x, q->Mall, q->C, q->loss, q->target, q->weight, q->loss_out, q->grad, q->nv);
}

__global__ __launch_bounds__(64) void cgl_counters_add_k(int* p, int n, int v) {
  if ((int)threadIdx.x < n) p[threadIdx.x] += v;
}

// Real-batch gather of the worker's sampler: dst[r] = src[idx ? idx[r] : row0 + r] (rows of
// row_floats floats; DataLoader(shuffle=True) over a device-resident shard, capgan.py:282,326-332).
__global__ __launch_bounds__(256) void cgl_gather_rows_k(const float* src, const int* idx, long row0, int nrows,
                                                         int rowf, float* dst) {
  const long n = (long)nrows * rowf;
  for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const int r = (int)(e / rowf), c = (int)(e - (long)r * rowf);
    const long sr = idx ? (long)gldi(idx + r) : row0 + r;
    gst(dst + e, gld(src + sr * rowf + c));
  }
}

// lambda-weighting of the gathered worker losses (cgl_weights of cgl_kernels.hip: capgan.py:247-248,
// mixed-gan.py:276, MDGAN/MNIST/mdgan.py:203, CGLGAN/2DMG/main.py:261-264) and scaling of this
// worker's exchange gradient by its alpha, before the all-reduce(sum) of the exchange.
struct CglWeightsArgs {
  int mode, n, rank;
  float lam;
  float beta[CGL_MAX_WORKERS];
  const float* losses;
  float* x;
  long nx;
  float* alpha_out;           // [n] (written by block 0), may be null
};

__global__ __launch_bounds__(256) void cgl_weights_scale_k(CglWeightsArgs a) {
  __shared__ float s_alpha;
  __shared__ float s_l[CGL_MAX_WORKERS], s_al[CGL_MAX_WORKERS], s_t[2][CGL_MAX_WORKERS];
  if (threadIdx.x == 0) {
    for (int q = 0; q < a.n; ++q) s_l[q] = gld(a.losses + q);
    cgl_weights(a.mode, a.n, a.lam, a.beta, s_l, s_al, s_t[0], s_t[1]);
    s_alpha = s_al[a.rank];
    if (blockIdx.x == 0 && a.alpha_out)
      for (int q = 0; q < a.n; ++q) gst(a.alpha_out + q, s_al[q]);
  }
  __syncthreads();
  const float al = s_alpha;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < a.nx; i += (long)gridDim.x * 256) gst(a.x + i, gld(a.x + i) * al);
}

// ==========================================================================================
// Host side: tap tables, launch planning, C ABI.
namespace {

struct ConvGeom {
  int n, h, w, cin, cout, stride, up, ks;   // ks: kernel size 3 (padding 1) or 1 (dense layer)
  int hv, wv, ho, wo;        // virtual (upsampled) input dims, output dims
};

int conv_geom(int n, int h, int w, int cin, int cout, int stride, int up, ConvGeom& g, int ks = 3) {
  if (n < 1 || h < 1 || w < 1 || cin < 1 || cout < 1 || (stride != 1 && stride != 2) || (up != 0 && up != 1))
    return CGL_E_ARG;
  if (up && stride != 1) return CGL_E_ARG;   // the reference only upsamples before stride-1 convs
  if (ks != 3 && (ks != 1 || stride != 1 || up)) return CGL_E_ARG;
  if (cin > 65536 || cout > 65536) return CGL_E_ARG;
  g.n = n; g.h = h; g.w = w; g.cin = cin; g.cout = cout; g.stride = stride; g.up = up; g.ks = ks;
  g.hv = h << up;
  g.wv = w << up;
  g.ho = (g.hv - 1) / stride + 1;
  g.wo = (g.wv - 1) / stride + 1;
  if ((long)n * g.ho * g.wo > (1L << 30) || (long)n * h * w > (1L << 30)) return CGL_E_ARG;
  return 0;
}

// one spatial dimension of a tap table: offsets and the kernel taps combined into each
struct Taps1 {
  int T, off[4], mask[4];
};

// forward, output parity ph of a 2x upsample + 3x3 conv (phase form), on the low-res input
Taps1 taps_up_fwd(int ph) {
  Taps1 t;
  t.T = 2;
  if (ph == 0) { t.off[0] = -1; t.mask[0] = 1; t.off[1] = 0; t.mask[1] = 6; }
  else { t.off[0] = 0; t.mask[0] = 3; t.off[1] = 1; t.mask[1] = 4; }
  return t;
}
Taps1 taps_1x1() {
  Taps1 t;
  t.T = 1; t.off[0] = 0; t.mask[0] = 1;
  return t;
}
Taps1 taps_direct(int sign) {   // sign +1: forward (offset kh - 1); -1: input gradient (offset 1 - kh)
  Taps1 t;
  t.T = 3;
  for (int k = 0; k < 3; ++k) { t.off[k] = sign * (k - 1); t.mask[k] = 1 << k; }
  return t;
}
// input gradient of a 2x upsample + 3x3 conv: dX[y] = sum_o dY[2y + o] Wc[o], o = -1..2
Taps1 taps_up_bwd() {
  Taps1 t;
  t.T = 4;
  const int off[4] = {-1, 0, 1, 2}, mask[4] = {4, 6, 3, 1};
  for (int k = 0; k < 4; ++k) { t.off[k] = off[k]; t.mask[k] = mask[k]; }
  return t;
}
// input gradient of a stride-2 3x3 conv, input parity p: dX[2y + p] = sum dY[y + o] W[kh]
Taps1 taps_s2_bwd(int p) {
  Taps1 t;
  if (p == 0) { t.T = 1; t.off[0] = 0; t.mask[0] = 2; }
  else { t.T = 2; t.off[0] = 0; t.mask[0] = 4; t.off[1] = 1; t.mask[1] = 1; }
  return t;
}

// Fill the geometry of one problem (everything but tiles / pointers).
void set_prob(CglConvProb& P, int nimg, int OH, int OW, int osy, int osx, int ooy, int oox, int YH, int YW, int ldy,
              int isy, int isx, int IH, int IW, int ish, int XH, int XW, int Cin, int N, const Taps1& ty,
              const Taps1& tx) {
  std::memset(&P, 0, sizeof(P));
  P.M = nimg * OH * OW;
  P.N = N;
  P.K = ty.T * tx.T * Cin;
  P.Kp = (P.K + 15) & ~15;
  P.OH = OH; P.OW = OW;
  P.osy = osy; P.osx = osx; P.ooy = ooy; P.oox = oox;
  P.YH = YH; P.YW = YW; P.ldy = ldy;
  P.isy = isy; P.isx = isx;
  P.IH = IH; P.IW = IW; P.ish = ish;
  P.XH = XH; P.XW = XW; P.Cin = Cin;
  P.Ty = ty.T; P.Tx = tx.T;
  for (int k = 0; k < 4; ++k) {
    P.dy[k] = k < ty.T ? ty.off[k] : 0;
    P.ym[k] = k < ty.T ? ty.mask[k] : 0;
    P.dx[k] = k < tx.T ? tx.off[k] : 0;
    P.xm[k] = k < tx.T ? tx.mask[k] : 0;
  }
}

// Problems of a forward conv (output = Y [n][ho][wo][cout], input X [n][h][w][cin]).
int fwd_probs(const ConvGeom& g, CglConvProb* P) {
  if (g.ks == 1) {
    set_prob(P[0], g.n, g.h, g.w, 1, 1, 0, 0, g.h, g.w, g.cout, 1, 1, g.h, g.w, 0, g.h, g.w, g.cin, g.cout, taps_1x1(),
             taps_1x1());
    return 1;
  }
  if (g.up) {
    int np = 0;
    for (int ph = 0; ph < 2; ++ph)
      for (int pw = 0; pw < 2; ++pw)
        set_prob(P[np++], g.n, g.h, g.w, 2, 2, ph, pw, g.ho, g.wo, g.cout, 1, 1, g.h, g.w, 0, g.h, g.w, g.cin, g.cout,
                 taps_up_fwd(ph), taps_up_fwd(pw));
    return np;
  }
  set_prob(P[0], g.n, g.ho, g.wo, 1, 1, 0, 0, g.ho, g.wo, g.cout, g.stride, g.stride, g.h, g.w, 0, g.h, g.w, g.cin,
           g.cout, taps_direct(1), taps_direct(1));
  return 1;
}

// Problems of the input gradient (output = dX [n][h][w][cin], input dY [n][ho][wo][cout]).
int bwd_probs(const ConvGeom& g, CglConvProb* P) {
  if (g.ks == 1) {
    set_prob(P[0], g.n, g.h, g.w, 1, 1, 0, 0, g.h, g.w, g.cin, 1, 1, g.h, g.w, 0, g.h, g.w, g.cout, g.cin, taps_1x1(),
             taps_1x1());
    return 1;
  }
  if (g.up) {
    set_prob(P[0], g.n, g.h, g.w, 1, 1, 0, 0, g.h, g.w, g.cin, 2, 2, g.ho, g.wo, 0, g.ho, g.wo, g.cout, g.cin,
             taps_up_bwd(), taps_up_bwd());
    return 1;
  }
  if (g.stride == 1) {
    set_prob(P[0], g.n, g.h, g.w, 1, 1, 0, 0, g.h, g.w, g.cin, 1, 1, g.ho, g.wo, 0, g.ho, g.wo, g.cout, g.cin,
             taps_direct(-1), taps_direct(-1));
    return 1;
  }
  int np = 0;
  for (int py = 0; py < 2; ++py)
    for (int px = 0; px < 2; ++px) {
      const int OH = (g.h - py + 1) / 2, OW = (g.w - px + 1) / 2;
      if (OH < 1 || OW < 1) continue;
      set_prob(P[np++], g.n, OH, OW, 2, 2, py, px, g.h, g.w, g.cin, 1, 1, g.ho, g.wo, 0, g.ho, g.wo, g.cout, g.cin,
               taps_s2_bwd(py), taps_s2_bwd(px));
    }
  return np;
}

inline int64_t al256(int64_t b) { return (b + 255) & ~int64_t(255); }

// MFMA tiling of a forward / input-gradient launch: (TM, TN) 32x32 blocks per wave, WM x WN waves
// over the output tile, WK waves splitting K.  Large problems: 2x2 blocks, waves along N when
// N > 64; problems that would give fewer than ~512 workgroups shrink the tile and split K inside
// the workgroup (LDS reduction) so every CU gets work.
struct ConvTiling { int TM, TN, WM, WN, WK; };
ConvTiling conv_tiling(int N) {
  if (N > 64) return {2, 2, 2, 2, 1};      // 128 x 128
  if (N > 32) return {2, 2, 4, 1, 1};      // 256 x 64
  return {2, 1, 4, 1, 1};                  // 256 x 32
}

long conv_wgs(const CglConvProb* P, int np, const ConvTiling& t) {
  long wg = 0;
  for (int i = 0; i < np; ++i)
    wg += (long)((P[i].M + 32 * t.TM * t.WM - 1) / (32 * t.TM * t.WM)) *
          ((P[i].N + 32 * t.TN * t.WN - 1) / (32 * t.TN * t.WN));
  return wg;
}

ConvTiling conv_tiling_for(const CglConvProb* P, int np) {
  ConvTiling t = conv_tiling(P[0].N);
  if (conv_wgs(P, np, t) >= 512) return t;
  const ConvTiling mid = {2, P[0].N > 32 ? 2 : 1, 1, 1, 4};   // 64 x 64 (64 x 32), K split 4 ways
  if (conv_wgs(P, np, mid) >= 512) return mid;
  return {1, 1, 1, 1, 4};                                    // 32 x 32, K split 4 ways
}

int64_t packed_floats(const CglConvProb* P, int np) {
  int64_t t = 0;
  for (int i = 0; i < np; ++i) t += al256((int64_t)P[i].N * P[i].Kp * 4) / 4;
  return t;
}

struct WgradPlan {
  CglConvProb P[CGL_CONV_MAXP];
  int np;
  ConvTiling t;
  int64_t part_floats;
};

// Weight-gradient plan: per-wave result tiles of (32 TM) x (32 TN) (rows = cout, cols = im2col
// columns); pixel splits so that all problems together give ~4096 wave units, each covering >= 32
// chunks of 16 pixels, with the partial tiles capped at 8M floats (32 MB).
// the input-stationary one-output-channel weight gradient (cgl_conv_wgrad_n1t) applies
bool wgrad_n1t_ok(const ConvGeom& g, const CglConvProb& P0) {
  const int c4 = P0.Cin / 4;
  return g.cout == 1 && g.stride == 1 && !g.up && P0.Cin % 4 == 0 && c4 >= 1 && c4 <= 64 && (c4 & (c4 - 1)) == 0 &&
         P0.Ty * P0.Tx <= 16 && (256 / c4) * P0.Ty * P0.Tx * P0.Cin <= 16384;
}

// the MFMA weight gradient also produces the bias gradient, from an im2col column of ones (column K)
// when the column is free (K is not a multiple of the tile width, so it lands in padding) or the
// layer is small (latency-bound: the extra tile costs less than the two column-sum launches); the
// vector one-output-channel kernels keep the column sum
bool wgrad_bias_col(const ConvGeom& g, const CglConvProb* P, int np) {
  if (g.cout == 1 && np == 1) return false;
  const int tw = P[0].K > 32 ? 64 : 32;
  int64_t macs = 0;
  bool free_col = true;
  for (int i = 0; i < np; ++i) {
    macs += (int64_t)P[i].M * P[i].N * P[i].K;
    free_col = free_col && (P[i].K % tw != 0);
  }
  return free_col || macs < ((int64_t)1 << 28);
}

WgradPlan wgrad_plan(const ConvGeom& g, bool bias = true) {
  WgradPlan w;
  w.np = fwd_probs(g, w.P);
  const int wb = bias && wgrad_bias_col(g, w.P, w.np) ? 1 : 0;
  w.t = ConvTiling{g.cout > 32 ? 2 : 1, w.P[0].K + wb > 32 ? 2 : 1, 1, 1, 1};
  int tiles_total = 0;
  int64_t nk_total = 0;
  for (int i = 0; i < w.np; ++i) {
    CglConvProb& P = w.P[i];
    P.Kp = (P.K + wb + 15) & ~15;   // partial row length (room for the bias column)
    P.tiles_m = (P.N + 32 * w.t.TM - 1) / (32 * w.t.TM);
    P.tiles_n = (P.K + wb + 32 * w.t.TN - 1) / (32 * w.t.TN);
    tiles_total += P.tiles_m * P.tiles_n;
    nk_total += (int64_t)P.N * P.Kp;
  }
  static const int wg_units = getenv("CGL_WG_UNITS") ? atoi(getenv("CGL_WG_UNITS")) : 2048;
  int s = std::max(1, wg_units / std::max(1, tiles_total));
  s = (int)std::min<int64_t>(s, std::max<int64_t>(1, (8 << 20) / std::max<int64_t>(1, nk_total)));
  w.part_floats = 0;
  for (int i = 0; i < w.np; ++i) {
    CglConvProb& P = w.P[i];
    const int nchk = (P.M + 15) / 16;
    P.splits = std::max(1, std::min(std::min(s, nchk / 4), 1024));
    if (g.cout == 1 && w.np == 1)   // vector kernels: >= 256 (input-stationary) / 32 pixels per split
      P.splits = std::max(1, std::min(1024, P.M / (wgrad_n1t_ok(g, P) ? 256 : 32)));
    w.part_floats += al256((int64_t)P.splits * P.N * P.Kp * 4) / 4;
  }
  return w;
}

int64_t conv_ws_bytes(const ConvGeom& g) {
  CglConvProb P[CGL_CONV_MAXP];
  int64_t a = packed_floats(P, fwd_probs(g, P));
  int64_t b = packed_floats(P, bwd_probs(g, P));
  WgradPlan w = wgrad_plan(g);
  const int64_t bias_part = al256(((int64_t)g.n * g.ho * g.wo + 31) / 32 * g.cout * 16) / 4 + 64;
  return 4 * (std::max(a, b) + w.part_floats + 2 * bias_part) + 4096;
}

// Packed-operand layout of one op (the problems of fwd_probs / bwd_probs): problem i's [N][Kp]
// block at base + (256-byte aligned running offset).  Returns the total floats.
int64_t pack_layout(CglConvProb* P, int np, const float* base) {
  int64_t off = 0;
  for (int i = 0; i < np; ++i) {
    P[i].Wp = base ? base + off : nullptr;
    off += al256((int64_t)P[i].N * P[i].Kp * 4) / 4;
  }
  return off;
}

int launch_pack(const float* W, const ConvGeom& g, int transpose, CglConvProb* P, int np, float* dst,
                hipStream_t s) {
  CglPackArgs a;
  std::memset(&a, 0, sizeof(a));
  a.W = W;
  a.cout = g.cout;
  a.cin = g.cin;
  a.transpose = transpose;
  a.np = np;
  a.ks = g.ks;
  int64_t off = 0;
  int64_t e = 0;
  for (int i = 0; i < np; ++i) {
    a.dst[i] = dst + off;
    P[i].Wp = dst + off;
    off += al256((int64_t)P[i].N * P[i].Kp * 4) / 4;
    a.N[i] = P[i].N;
    a.Kp[i] = P[i].Kp;
    a.Cg[i] = P[i].Cin;
    a.Tx[i] = P[i].Tx;
    a.T[i] = P[i].Ty * P[i].Tx;
    for (int k = 0; k < 4; ++k) { a.ym[i][k] = P[i].ym[k]; a.xm[i][k] = P[i].xm[k]; }
    a.begin[i] = (int)e;
    e += (int64_t)P[i].N * P[i].Kp;
  }
  a.begin[np] = (int)e;
  hipLaunchKernelGGL(cgl_conv_pack, dim3((unsigned)((e + 255) / 256)), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

// the vector one-output-channel kernel: Cin % 4 == 0, Cin / 4 a power of two (or a multiple of 64),
// at most 16 (tap, float4-block) pairs per lane
bool n1_ok(const CglConvProb* P, int np) {
  for (int i = 0; i < np; ++i) {
    const int c4 = P[i].Cin / 4;
    if (P[i].Cin % 4 || c4 < 1) return false;
    const int lanes = c4 < 64 ? c4 : 64;
    if ((lanes & (lanes - 1)) || c4 % lanes) return false;
    if (P[i].Ty * P[i].Tx * (c4 / lanes) > 16) return false;
  }
  return true;
}

struct StatBwd {
  const float* x = nullptr; const float* post = nullptr; const float* mean = nullptr; float slope = 0.f;
  const float* psc = nullptr; int psc_ld = 0;    // LeakyReLU'(post) from the forward's scale / shift (post null)
};

struct BnIn { const float* coef = nullptr; int groups = 1, gimg = 1, act = 0; float slope = 0.f; int g0 = 0; };

// The halo path: 4 problems over one input through one tile grid -- the output parities of an upsampling
// conv (2x2 taps, offsets within one pixel), 64 output channels (one 2x2-block wave tile), whole 64-row
// tiles of whole low-res rows per image, a window that fits 64 KB of LDS.
bool conv_halo_ok(const CglConvProb* P, int np) {
  if (np != 4) return false;
  const CglConvProb& a = P[0];
  if (a.OW < 1 || 64 % a.OW || (a.OH * a.OW) % 64 || a.M % 64 || a.Cin % 16 || (a.N != 64 && a.N != 128))
    return false;
  if ((64 / a.OW + 2) * (a.OW + 2) * (a.Cin + 4) * 4 > 65536) return false;
  for (int i = 0; i < np; ++i) {
    const CglConvProb& p = P[i];
    if (p.X != a.X || p.M != a.M || p.N != a.N || p.Cin != a.Cin || p.OH != a.OH || p.OW != a.OW || p.Ty != 2 ||
        p.Tx != 2 || p.isy != 1 || p.isx != 1 || p.ish != 0 || p.IH != a.OH || p.IW != a.OW || p.Kp != p.K)
      return false;
    for (int t = 0; t < 2; ++t)
      if (p.dy[t] < -1 || p.dy[t] > 1 || p.dx[t] < -1 || p.dx[t] > 1) return false;
  }
  return true;
}

int launch_conv_mma(CglConvProb* P, int np, const float* bias, int act, float slope, const float* drop,
                    hipStream_t s, double* st_part = nullptr, int st_cpg = 0, const StatBwd* sb = nullptr,
                    const BnIn* bi = nullptr, const int* st_nv = nullptr) {
  const int N = P[0].N;
  CglConvLaunch L;
  std::memset(&L, 0, sizeof(L));
  L.np = np;
  L.bias = bias;
  L.act = act;
  if (bi && bi->coef) {
    L.in_coef = bi->coef;
    L.in_groups = bi->groups;
    L.in_gimg = bi->gimg;
    L.in_act = bi->act;
    L.in_slope = bi->slope;
    if (bi->act == CGL_EPI_ACT_LEAKY && !(bi->slope > 0.f && bi->slope <= 1.f)) return CGL_E_ARG;   // (max form)
  }
  L.slope = slope;
  L.drop = drop;
  L.st_part = st_part;
  L.st_cpg = st_cpg;
  L.st_nv = st_nv;
  if (st_nv && (!st_part || sb || np != 1)) return CGL_E_ARG;   // forward statistics of one problem only
  if (sb) {
    L.st_mode = 1;
    L.st_x = sb->x;
    L.st_post = sb->post;
    L.st_psc = sb->psc;
    L.st_psc_ld = sb->psc_ld;
    L.st_mean = sb->mean;
    L.st_slope = sb->slope;
  }
  if (st_part && N == 1) return CGL_E_ARG;   // statistics only from the MFMA kernel
  if (N == 1 && np == 1 && P[0].Ty == 3 && P[0].Tx == 3 && P[0].isy == 1 && P[0].isx == 1 && P[0].ish == 0 &&
      P[0].osy == 1 && P[0].osx == 1 && P[0].dy[0] == -1 && P[0].dx[0] == -1 && P[0].Cin % 4 == 0 &&
      P[0].Cin <= 256 && ((P[0].Cin / 4) & (P[0].Cin / 4 - 1)) == 0 && P[0].XH == P[0].OH && P[0].XW == P[0].OW &&
      (CGL_N1T_TH + 2) * (P[0].OW + 2) * P[0].Cin * 4 <= 65536) {
    const int tiles_y = (P[0].OH + CGL_N1T_TH - 1) / CGL_N1T_TH;
    const int nimg = P[0].M / (P[0].OH * P[0].OW);
    L.p[0] = P[0];
    const int lds = (CGL_N1T_TH + 2) * (P[0].OW + 2) * P[0].Cin * 4;
    if (P[0].Cin == 64 && P[0].OW == 32 && P[0].YW == 32 && P[0].YH == P[0].OH && !getenv("CGL_N1_TILE")) {
      hipLaunchKernelGGL(cgl_conv_n1_part, dim3(nimg * ((P[0].OH + CGL_N1P_TH - 1) / CGL_N1P_TH)), dim3(256), 0, s, L);
      return (int)hipGetLastError();
    }
    if (L.in_coef) return CGL_E_ARG;     // the folded BatchNorm input: cgl_conv_n1_part and the MFMA kernels only
    if (P[0].Cin == 64 && P[0].OW == 32)
      hipLaunchKernelGGL((cgl_conv_n1_tile<16, 32>), dim3(nimg * tiles_y), dim3(256), lds, s, L);
    else
      hipLaunchKernelGGL((cgl_conv_n1_tile<0, 0>), dim3(nimg * tiles_y), dim3(256), lds, s, L);
    return (int)hipGetLastError();
  }
  if (L.in_coef && N == 1) return CGL_E_ARG;
  if (N == 1 && n1_ok(P, np)) {
    int wg = 0;
    for (int i = 0; i < np; ++i) {
      const int c4 = P[i].Cin / 4, lanes = c4 < 64 ? c4 : 64;
      const int per_wg = 4 * (64 / lanes) * CGL_N1_IT;
      P[i].wg_begin = wg;
      wg += (P[i].M + per_wg - 1) / per_wg;
      L.p[i] = P[i];
    }
    hipLaunchKernelGGL(cgl_conv_n1, dim3(wg), dim3(256), 0, s, L);
    return (int)hipGetLastError();
  }
  // the upsampling conv's 4 parity problems from one LDS-staged window per 64-row tile (CGL_CONV_HALO=0: off)
  const int halo_env = getenv("CGL_CONV_HALO") ? atoi(getenv("CGL_CONV_HALO")) : 1;   // read per launch (tests toggle it)
  if (halo_env && !L.st_mode && !L.st_nv && conv_halo_ok(P, np)) {
    const int lds = (64 / P[0].OW + 2) * (P[0].OW + 2) * (P[0].Cin + 4) * 4;
    L.WM = L.WN = L.WK = 1;
    for (int i = 0; i < np; ++i) {
      P[i].tiles_m = P[i].M / 64;
      P[i].tiles_n = N / 64;   // a workgroup per (64-row tile, 64-channel half); each stages the tile's window
      P[i].wg_begin = 0;
      L.p[i] = P[i];
    }
    const int grid = P[0].M / 64 * (N / 64);
    if (L.in_coef) hipLaunchKernelGGL((cgl_conv_fwd_halo<true>), dim3(grid), dim3(256), lds, s, L);
    else hipLaunchKernelGGL((cgl_conv_fwd_halo<false>), dim3(grid), dim3(256), lds, s, L);
    return (int)hipGetLastError();
  }
  const ConvTiling t = conv_tiling_for(P, np);
  L.WM = t.WM;
  L.WN = t.WN;
  L.WK = t.WK;
  int lds = t.WK > 1 ? (t.WK - 1) * t.WM * t.WN * t.TM * t.TN * 16 * 64 * 4 : 0;
  if (L.in_coef) lds += ((2 * L.in_groups * P[0].Cin + 63) & ~63) * 4;   // the staged scale / shift
  bool fast = true;
  int wg = 0;
  for (int i = 0; i < np; ++i) {
    P[i].tiles_m = (P[i].M + 32 * t.TM * t.WM - 1) / (32 * t.TM * t.WM);
    P[i].tiles_n = (P[i].N + 32 * t.TN * t.WN - 1) / (32 * t.TN * t.WN);
    P[i].wg_begin = wg;
    wg += P[i].tiles_m * P[i].tiles_n;
    fast = fast && (P[i].Cin % 16 == 0 || (P[i].Ty * P[i].Tx == 1 && P[i].Cin % 4 == 0));
    L.p[i] = P[i];
  }
  // interleaved tile order for problems that read one input through the same tile grid
  // (CGL_CONV_ILV=0: problem-major order)
  static const int ilv_env = getenv("CGL_CONV_ILV") ? atoi(getenv("CGL_CONV_ILV")) : 1;
  L.ilv = ilv_env != 0 && np > 1;
  for (int i = 1; i < np; ++i)
    L.ilv = L.ilv && P[i].X == P[0].X && P[i].tiles_m == P[0].tiles_m && P[i].tiles_n == P[0].tiles_n;
  if (L.in_coef) {
    for (int i = 0; i < np; ++i)
      if (P[i].Cin != P[0].Cin || P[i].Cin > 512) return CGL_E_ARG;
    if (!fast) return CGL_E_ARG;
    if (t.TM == 2 && t.TN == 2) hipLaunchKernelGGL((cgl_conv_fwd<2, 2, true, true>), dim3(wg), dim3(256), lds, s, L);
    else if (t.TM == 2) hipLaunchKernelGGL((cgl_conv_fwd<2, 1, true, true>), dim3(wg), dim3(256), lds, s, L);
    else hipLaunchKernelGGL((cgl_conv_fwd<1, 1, true, true>), dim3(wg), dim3(256), lds, s, L);
    return (int)hipGetLastError();
  }
  // the 2 x 2-wave 128 x 128 tiling of a FAST problem: LDS-staged operand panels (CGL_CONV_LDSM=0: the direct
  // loads; bitwise the same results)
  const int ldsm_env = getenv("CGL_CONV_LDSM") ? atoi(getenv("CGL_CONV_LDSM")) : 1;   // (per launch: tests toggle it)
  if (t.TM == 2 && t.TN == 2 && fast && ldsm_env && t.WM == 2 && t.WN == 2 && t.WK == 1) {
    hipLaunchKernelGGL((cgl_conv_fwd<2, 2, true, false, true>), dim3(wg), dim3(256), 2 * 2 * 128 * 20 * 4, s, L);
  } else if (t.TM == 2 && t.TN == 2) {
    if (fast) hipLaunchKernelGGL((cgl_conv_fwd<2, 2, true>), dim3(wg), dim3(256), lds, s, L);
    else hipLaunchKernelGGL((cgl_conv_fwd<2, 2, false>), dim3(wg), dim3(256), lds, s, L);
  } else if (t.TM == 2) {
    if (fast) hipLaunchKernelGGL((cgl_conv_fwd<2, 1, true>), dim3(wg), dim3(256), lds, s, L);
    else hipLaunchKernelGGL((cgl_conv_fwd<2, 1, false>), dim3(wg), dim3(256), lds, s, L);
  } else {
    if (fast) hipLaunchKernelGGL((cgl_conv_fwd<1, 1, true>), dim3(wg), dim3(256), lds, s, L);
    else hipLaunchKernelGGL((cgl_conv_fwd<1, 1, false>), dim3(wg), dim3(256), lds, s, L);
  }
  return (int)hipGetLastError();
}


int fin_nocache() {
  static const int v = getenv("CGL_FIN_NOCACHE") ? atoi(getenv("CGL_FIN_NOCACHE")) : 0;
  return v;
}

// Rows per channel-reduction chunk (one workgroup each): 128, halved down to 32 while a BatchNorm call would
// get fewer than 64 chunks -- the discriminator's 2 x 2 and 4 x 4 maps (1024-4096 rows per call) otherwise ran
// their reduction on 8-32 workgroups, latency-bound (CGL_CHAN_MINCH=0: plain 128).
int chan_chunk(int64_t gr) {
  static const int minch = getenv("CGL_CHAN_MINCH") ? atoi(getenv("CGL_CHAN_MINCH")) : 64;
  int R = 128;
  while (R > 1 && gr % R != 0) R >>= 1;
  while (R > 32 && gr / R < minch && gr % (R >> 1) == 0) R >>= 1;
  return R;
}

bool pow2_le256(int C) { return C >= 1 && C <= 256 && (C & (C - 1)) == 0; }

// per-column sum of X [rows][C] into out[C] (bias gradient): chunk partials (double), then a
// fixed-order sum over chunks (cgl_bn_finalize mode 2)
// the column sums' partial pass (launched) and their finalize's arguments (f: launched by the caller)
int col_sum_part(const float* X, int64_t rows, int C, double* part, float* out, hipStream_t s, CglBnFinArgs& f) {
  int nch;
  if (pow2_le256(C)) {
    const int R = 256;
    nch = (int)((rows + R - 1) / R);
    CglChanArgs a;
    std::memset(&a, 0, sizeof(a));
    a.X = X; a.rows = (int)rows; a.C = C; a.R = R; a.mode = 2; a.gr = (int)rows; a.part = part;
    launch_chan_reduce(a, nch, s);
  } else {
    const int R = 32;
    nch = (int)((rows + R - 1) / R);
    hipLaunchKernelGGL(cgl_colsum_k, dim3((C + 255) / 256, nch), dim3(256), 0, s, X, (int)rows, C, R, part);
  }
  std::memset(&f, 0, sizeof(f));
  f.part = part; f.C = C; f.groups = 1; f.chunks_per_group = nch; f.mode = 2; f.dgamma = out;
  f.nocache = fin_nocache();
  return (int)hipGetLastError();
}

int col_sum(const float* X, int64_t rows, int C, double* part, float* out, hipStream_t s) {
  CglBnFinArgs f;
  const int rc = col_sum_part(X, rows, C, part, out, s, f);
  if (rc) return rc;
  hipLaunchKernelGGL(cgl_bn_finalize, dim3(C), dim3(256), 0, s, f);
  return (int)hipGetLastError();
}

}  // namespace

namespace {

// BatchNorm statistics in the forward epilogue: supported when every problem's rows per forward
// call are whole 32-row chunks and the launch takes the MFMA kernel; returns the chunks per call
// (0: unsupported)
int stat_chunks_per_group(const ConvGeom& g, int groups, int bwd = 0) {
  if (groups < 1 || g.n % groups || (bwd ? g.cin : g.cout) < 32) return 0;
  if (bwd && g.cout == 1) return 0;   // the vector one-output-channel input gradient has no epilogue
  CglConvProb P[CGL_CONV_MAXP];
  const int np = bwd ? bwd_probs(g, P) : fwd_probs(g, P);
  int cpg = 0;
  for (int i = 0; i < np; ++i) {
    const long gr = (long)(g.n / groups) * P[i].OH * P[i].OW;
    if (gr % 32) return 0;
    cpg += (int)(gr / 32);
  }
  return cpg;
}

// the vector one-input-channel kernels (cgl_conv_c1_*) apply
bool c1_ok(const ConvGeom& g) {
  return g.cin == 1 && g.ks == 3 && !g.up && g.cout % 4 == 0 && g.cout <= 16 && 256 % g.cout == 0;
}

int conv_fwd_impl(const ConvGeom& g, const float* X, const float* W, const float* bias, float* Y, int act, float slope,
                  const float* drop, void* ws, int64_t wsb, hipStream_t s, const float* Wp = nullptr,
                  double* st_part = nullptr, int st_groups = 1, const BnIn* bi = nullptr, const int* st_nv = nullptr) {
  if (!X || !(W || Wp) || !Y || !ws || act < 0 || act > 3 || !al16(ws) || (Wp && !al16(Wp))) return CGL_E_ARG;
  if (wsb < conv_ws_bytes(g)) return CGL_E_SIZE;
  if ((g.cin % 4 == 0) && !al16(X)) return CGL_E_ARG;
  CglConvProb P[CGL_CONV_MAXP];
  const int np = fwd_probs(g, P);
  int cpg = 0;
  if (st_part) {
    if (!(cpg = stat_chunks_per_group(g, st_groups)) || ((uintptr_t)st_part & 15)) return CGL_E_ARG;
    int off = 0;
    for (int i = 0; i < np; ++i) {
      P[i].st_gr = (g.n / st_groups) * P[i].OH * P[i].OW;
      P[i].st_off = off;
      off += P[i].st_gr / 32;
    }
  }
  for (int i = 0; i < np; ++i) {
    P[i].X = X;
    P[i].Y = Y;
  }
  if (bi && bi->coef && (!Wp || bi->groups < 1 || g.n % bi->groups || !al16(bi->coef) || g.cin % 4 ||
                         (bi->act != CGL_EPI_ACT_NONE && bi->act != CGL_EPI_ACT_LEAKY)))
    return CGL_E_ARG;
  if (c1_ok(g) && !st_part && !(bi && bi->coef) && act != CGL_EPI_ACT_TANH && act != CGL_EPI_ACT_SIGMOID && al16(Y) &&
      (!drop || al16(drop))) {
    // the packed forward operand of a Cin = 1 conv is [cout][16] (9 taps, zero padded)
    CglC1Args a;
    std::memset(&a, 0, sizeof(a));
    a.X = X; a.W = Wp ? Wp : W; a.wst = Wp ? 16 : 9; a.bias = bias; a.Y = Y; a.drop = drop;
    a.n = g.n; a.h = g.h; a.w = g.w; a.ho = g.ho; a.wo = g.wo; a.cout = g.cout; a.stride = g.stride;
    a.act = act; a.slope = slope;
    const long npix = (long)g.n * g.ho * g.wo;
    hipLaunchKernelGGL(cgl_conv_c1_fwd, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, s, a);
    return (int)hipGetLastError();
  }
  int rc;
  if (Wp) pack_layout(P, np, Wp);
  else if ((rc = launch_pack(W, g, 0, P, np, (float*)ws, s))) return rc;
  return launch_conv_mma(P, np, bias, act, slope, drop, s, st_part, cpg, nullptr, bi, st_nv);
}

int conv_bwd_data_impl(const ConvGeom& g, const float* dY, const float* W, float* dX, void* ws, int64_t wsb,
                       hipStream_t s, const float* Wp = nullptr, double* st_part = nullptr, int st_groups = 1,
                       const StatBwd* sb = nullptr) {
  if (!dY || !(W || Wp) || !dX || !ws || !al16(ws) || (Wp && !al16(Wp))) return CGL_E_ARG;
  if (wsb < conv_ws_bytes(g)) return CGL_E_SIZE;
  if ((g.cout % 4 == 0) && !al16(dY)) return CGL_E_ARG;
  int cpg = 0;
  if (st_part) {
    if (!sb || !sb->x || !sb->mean || !(cpg = stat_chunks_per_group(g, st_groups, 1)) || ((uintptr_t)st_part & 15))
      return CGL_E_ARG;
  }
  if (!st_part && W && g.cout == 1 && g.cin == 64 && g.ks == 3 && g.stride == 1 && !g.up && al16(dX) &&
      (int64_t)g.n * g.h * g.w < (int64_t)1 << 30) {
    const int npix = g.n * g.h * g.w;
    hipLaunchKernelGGL((cgl_conv_bwd_n1<16>), dim3((npix + 16 * CGL_BN1_PPT - 1) / (16 * CGL_BN1_PPT)), dim3(256), 0, s, dY, W, dX, npix, g.h, g.w,
                       CglN1Stats{});
    return (int)hipGetLastError();
  }
  CglConvProb P[CGL_CONV_MAXP];
  const int np = bwd_probs(g, P);
  int off = 0;
  for (int i = 0; i < np; ++i) {
    P[i].X = dY;
    P[i].Y = dX;
    if (st_part) {
      P[i].st_gr = (g.n / st_groups) * P[i].OH * P[i].OW;
      P[i].st_off = off;
      off += P[i].st_gr / 32;
    }
  }
  int rc;
  if (Wp) pack_layout(P, np, Wp);
  else if ((rc = launch_pack(W, g, 1, P, np, (float*)ws, s))) return rc;
  return launch_conv_mma(P, np, nullptr, CGL_EPI_ACT_NONE, 0.f, nullptr, s, st_part, cpg, st_part ? sb : nullptr);
}

// the ROW fast path of cgl_conv_wgrad_body: whole 8-pixel row segments in every problem
bool wgrad_row_ok(const WgradPlan& pl) {
  for (int i = 0; i < pl.np; ++i)
    if (pl.P[i].OW % 8 != 0 || pl.P[i].M % 16 != 0) return false;
  return true;
}

// cgl_conv_wgrad_lds applies: no bias column, whole R x C tiles (N % R == 0, K % C == 0), 16-byte operand
// rows (Cin % 4 == 0 so 4 columns are one tap, ldy % 4 == 0, aligned bases), whole 16-pixel chunks inside one
// image (power-of-two output grids of >= 16 pixels: shift / mask decode), an unshifted input.  Returns WM (WN = 4 / WM), 0 = not applicable.
// CGL_WGRAD_LDS=0 keeps the wave-unit kernel (A/B).
int wgrad_lds_wm(const WgradPlan& pl, bool bias_col, const float* dY, const float* X) {
  static const int env = getenv("CGL_WGRAD_LDS") ? atoi(getenv("CGL_WGRAD_LDS")) : 1;
  if (!env || bias_col || !al16(dY) || !al16(X)) return 0;
  const int N = pl.P[0].N, K = pl.P[0].K;
  const int wm = (N % 128 == 0 && K % 128 == 0) ? 2 : ((N % 64 == 0 && K % 256 == 0) ? 1 : 0);
  if (!wm) return 0;
  for (int i = 0; i < pl.np; ++i) {
    const CglConvProb& P = pl.P[i];
    if (P.N != N || P.K != K || P.Cin % 4 || P.ldy % 4 || P.M % 16 || P.M < 16 * 64 || P.ish != 0) return 0;
    if ((P.OW & (P.OW - 1)) || (P.OH & (P.OH - 1)) || P.OW * P.OH < 16) return 0;
  }
  return wm;
}

// bi (may be null): X is the PRE-BatchNorm map of one forward call, applied in the operand loads -- only the
// LDS-staged MFMA weight gradient and the input-stationary one-output-channel one take it (CGL_E_ARG otherwise)
// Deferred weight-gradient reductions (cgl_conv_wgrad_defer_begin / _end): while open on the calling thread, a
// weight gradient launches its MFMA kernel and records its split reduction (or the c1 kernel's finish) here;
// _end launches every recorded one as one cgl_conv_wgrad_reduce_multi.
struct WgradDefer {
  bool on = false;
  CglWgradReduceMulti m{};
  bool has_c1 = false;
  bool add_fin(const CglBnFinArgs& f) {
    if (m.nfin >= CGL_WDEFER_FIN) return false;
    m.fin[m.nfin] = f;
    m.fbeg[m.nfin + 1] = m.fbeg[m.nfin] + f.C;
    ++m.nfin;
    return true;
  }
};
thread_local WgradDefer t_wdefer;

int conv_bwd_weight_impl(const ConvGeom& g, const float* dY, const float* X, float* dW, float* db, void* ws,
                         int64_t wsb, hipStream_t s, const BnIn* bi = nullptr, const float* ad_post = nullptr,
                         const float* ad_drop = nullptr, float ad_slope = 0.f) {
  if (!dY || !X || !dW || !ws || !al16(ws)) return CGL_E_ARG;
  if (wsb < conv_ws_bytes(g)) return CGL_E_SIZE;
  if (bi && (!bi->coef || !al16(bi->coef) || bi->g0 < 0 || bi->g0 >= bi->groups || g.cin % 4)) return CGL_E_ARG;
  if (g.cout > CGL_ZERO_PAGE || g.cin > CGL_ZERO_PAGE) return CGL_E_ARG;   // cgl_zero_page bound
  if (c1_ok(g)) {
    if (bi) return CGL_E_ARG;
    const long npix = (long)g.n * g.ho * g.wo;
    CglC1Args a;
    std::memset(&a, 0, sizeof(a));
    a.X = X; a.dY = dY; a.dW = dW; a.db = db;
    a.post = ad_post; a.drop = ad_drop; a.slope = ad_slope;
    a.n = g.n; a.h = g.h; a.w = g.w; a.ho = g.ho; a.wo = g.wo; a.cout = g.cout; a.stride = g.stride;
    a.chunk = 128;
    a.nblk = (int)((npix + a.chunk - 1) / a.chunk);
    if ((int64_t)a.nblk * g.cout * 10 * 4 > wsb) return CGL_E_SIZE;
    a.part = (float*)ws;
    hipLaunchKernelGGL(cgl_conv_c1_wgrad, dim3(a.nblk), dim3(256), 0, s, a);
    if (t_wdefer.on && !t_wdefer.has_c1) {   // the finish rides in the deferred reductions' launch
      t_wdefer.m.c1 = a;
      t_wdefer.m.c1_blocks = g.cout * 10;
      t_wdefer.has_c1 = true;
      return (int)hipGetLastError();
    }
    hipLaunchKernelGGL(cgl_conv_c1_wgrad_fin, dim3(g.cout * 10), dim3(256), 0, s, a);
    return (int)hipGetLastError();
  }
  WgradPlan pl = wgrad_plan(g, db != nullptr);
  const bool bias_col = db && wgrad_bias_col(g, pl.P, pl.np);
  CglConvLaunch L;
  std::memset(&L, 0, sizeof(L));
  L.np = pl.np;
  L.wbias = bias_col ? 1 : 0;
  L.WM = 1;
  L.WN = 1;
  L.WK = 1;
  if (bi) {
    L.in_coef = bi->coef;
    L.in_groups = bi->groups;
    L.in_gimg = bi->gimg;
    L.in_act = bi->act;
    L.in_slope = bi->slope;
    if (bi->act == CGL_EPI_ACT_LEAKY && !(bi->slope > 0.f && bi->slope <= 1.f)) return CGL_E_ARG;   // (max form)
    L.in_g0 = bi->g0;
  }
  float* part = (float*)ws;
  const bool valu = g.cout == 1 && pl.np == 1;   // cgl_conv_wgrad_n1 (splits set by wgrad_plan)
  const bool n1t = valu && wgrad_n1t_ok(g, pl.P[0]);
  int wg = 0;
  CglWgradReduceArgs r;
  std::memset(&r, 0, sizeof(r));
  r.dW = dW;
  r.cout = g.cout;
  r.cin = g.cin;
  r.np = pl.np;
  r.ks = g.ks;
  for (int i = 0; i < pl.np; ++i) {
    CglConvProb& P = pl.P[i];
    P.X = X;
    P.Y = (float*)dY;
    P.part = part;
    part += al256((int64_t)P.splits * P.N * P.Kp * 4) / 4;
    P.wg_begin = wg;
    wg += (P.tiles_m * P.tiles_n * P.splits + 3) / 4;   // 4 wave units per workgroup
    L.p[i] = P;
    r.part[i] = P.part;
    r.Kp[i] = P.Kp;
    r.K[i] = P.K;
    r.splits[i] = P.splits;
    r.Tx[i] = P.Tx;
    r.Ty[i] = P.Ty;
    for (int k = 0; k < 4; ++k) { r.ym[i][k] = P.ym[k]; r.xm[i][k] = P.xm[k]; }
  }
  const int lwm = valu ? 0 : wgrad_lds_wm(pl, bias_col, dY, X);
  if (bi && bi->gimg < g.n && (lwm || valu)) return CGL_E_ARG;   // stacked calls: the wave-unit kernel only
  if (lwm) {
    // workgroup tiles of 64 lwm x 256 / lwm over the plan's pixel splits (partials as sized by wgrad_plan);
    // CGL_WGRAD_KS = 2: two-half workgroups over half as many (twice as long) splits.  Measured neutral
    // (profiles/r04_conv_wgrad_ks_dfold.txt: the reduce gains 6.4 us per round, the two kernels lose 7.9 us),
    // so opt-in
    static const int ks = getenv("CGL_WGRAD_KS") && atoi(getenv("CGL_WGRAD_KS")) == 2 ? 2 : 1;
    int wgl = 0;
    for (int i = 0; i < pl.np; ++i) {
      CglConvProb& P = L.p[i];
      P.tiles_m = P.N / (64 * lwm);
      P.tiles_n = P.K / (256 / lwm);
      P.splits = std::max(1, P.splits / ks);
      r.splits[i] = P.splits;
      P.wg_begin = wgl;
      wgl += P.tiles_m * P.tiles_n * P.splits;
    }
    if (bi) {
      if (lwm == 2) hipLaunchKernelGGL((cgl_conv_wgrad_lds<2, 2, 1, true>), dim3(wgl), dim3(256), 0, s, L);
      else hipLaunchKernelGGL((cgl_conv_wgrad_lds<1, 4, 1, true>), dim3(wgl), dim3(256), 0, s, L);
    } else if (ks == 2) {
      if (lwm == 2) hipLaunchKernelGGL((cgl_conv_wgrad_lds<2, 2, 2>), dim3(wgl), dim3(512), 0, s, L);
      else hipLaunchKernelGGL((cgl_conv_wgrad_lds<1, 4, 2>), dim3(wgl), dim3(512), 0, s, L);
    } else {
      if (lwm == 2) hipLaunchKernelGGL((cgl_conv_wgrad_lds<2, 2, 1>), dim3(wgl), dim3(256), 0, s, L);
      else hipLaunchKernelGGL((cgl_conv_wgrad_lds<1, 4, 1>), dim3(wgl), dim3(256), 0, s, L);
    }
  }
  else if (bi && valu && !(n1t && pl.P[0].Cin == 64 && pl.P[0].XW == 32 && pl.P[0].XH == 32 &&
                          pl.P[0].Ty * pl.P[0].Tx == 9))
    return CGL_E_ARG;
  else if (bi && !valu) {
    // the wave-unit MFMA weight gradient with the BatchNorm applied per loaded value (up to two groups)
    if (bi->groups - bi->g0 > 2 && bi->gimg < g.n) return CGL_E_ARG;
    if (wgrad_row_ok(pl)) {
      if (pl.t.TM == 2 && pl.t.TN == 2) hipLaunchKernelGGL((cgl_conv_wgrad<2, 2, true, true>), dim3(wg), dim3(256), 0, s, L);
      else if (pl.t.TN == 2) hipLaunchKernelGGL((cgl_conv_wgrad<1, 2, true, true>), dim3(wg), dim3(256), 0, s, L);
      else if (pl.t.TM == 2) hipLaunchKernelGGL((cgl_conv_wgrad<2, 1, true, true>), dim3(wg), dim3(256), 0, s, L);
      else hipLaunchKernelGGL((cgl_conv_wgrad<1, 1, true, true>), dim3(wg), dim3(256), 0, s, L);
    } else if (pl.t.TM == 2 && pl.t.TN == 2) hipLaunchKernelGGL((cgl_conv_wgrad<2, 2, false, true>), dim3(wg), dim3(256), 0, s, L);
    else if (pl.t.TN == 2) hipLaunchKernelGGL((cgl_conv_wgrad<1, 2, false, true>), dim3(wg), dim3(256), 0, s, L);
    else if (pl.t.TM == 2) hipLaunchKernelGGL((cgl_conv_wgrad<2, 1, false, true>), dim3(wg), dim3(256), 0, s, L);
    else hipLaunchKernelGGL((cgl_conv_wgrad<1, 1, false, true>), dim3(wg), dim3(256), 0, s, L);
  }
  else if (n1t)
  {
    if (pl.P[0].Cin == 64 && pl.P[0].XW == 32 && pl.P[0].XH == 32 && pl.P[0].Ty * pl.P[0].Tx == 9)
    {
      const CglConvProb& P0 = pl.P[0];
      const long per_block = ((long)(P0.M / (P0.OH * P0.OW)) * P0.XH * P0.XW + P0.splits - 1) / P0.splits;
      const bool stage = P0.YH == P0.OH && P0.YW == P0.OW && P0.ldy == 1 && P0.OH == 32 && P0.OW == 32 &&
                         per_block + 2 * P0.OW + 2 <= 512;
      // one pixel per slot and step, dY window in LDS: 105 -> 57 us for the B=256 G Conv2d(64, 1)
      // (two / four pixels per step: 77 / 119 us; no staging: 90 us)
      if (bi && stage)
        hipLaunchKernelGGL((cgl_conv_wgrad_n1t<16, 32, 32, 1, 9216, 512, true>), dim3(P0.splits), dim3(256), 0, s, L);
      else if (bi)
        hipLaunchKernelGGL((cgl_conv_wgrad_n1t<16, 32, 32, 1, 9216, 0, true>), dim3(P0.splits), dim3(256), 0, s, L);
      else if (stage)
        hipLaunchKernelGGL((cgl_conv_wgrad_n1t<16, 32, 32, 1, 9216, 512>), dim3(P0.splits), dim3(256), 0, s, L);
      else hipLaunchKernelGGL((cgl_conv_wgrad_n1t<16, 32, 32, 1, 9216, 0>), dim3(P0.splits), dim3(256), 0, s, L);
    }
    else
      hipLaunchKernelGGL((cgl_conv_wgrad_n1t<0, 0, 0, 2, 16384, 0>), dim3(pl.P[0].splits), dim3(256), 0, s, L);
  }
  else if (valu)
    hipLaunchKernelGGL(cgl_conv_wgrad_n1, dim3((pl.P[0].K + 255) / 256, pl.P[0].splits), dim3(256), 0, s, L);
  else if (wgrad_row_ok(pl)) {
    if (pl.t.TM == 2 && pl.t.TN == 2) hipLaunchKernelGGL((cgl_conv_wgrad<2, 2, true>), dim3(wg), dim3(256), 0, s, L);
    else if (pl.t.TN == 2) hipLaunchKernelGGL((cgl_conv_wgrad<1, 2, true>), dim3(wg), dim3(256), 0, s, L);
    else if (pl.t.TM == 2) hipLaunchKernelGGL((cgl_conv_wgrad<2, 1, true>), dim3(wg), dim3(256), 0, s, L);
    else hipLaunchKernelGGL((cgl_conv_wgrad<1, 1, true>), dim3(wg), dim3(256), 0, s, L);
  }
  else if (pl.t.TM == 2 && pl.t.TN == 2) hipLaunchKernelGGL((cgl_conv_wgrad<2, 2>), dim3(wg), dim3(256), 0, s, L);
  else if (pl.t.TN == 2) hipLaunchKernelGGL((cgl_conv_wgrad<1, 2>), dim3(wg), dim3(256), 0, s, L);
  else if (pl.t.TM == 2) hipLaunchKernelGGL((cgl_conv_wgrad<2, 1>), dim3(wg), dim3(256), 0, s, L);
  else hipLaunchKernelGGL((cgl_conv_wgrad<1, 1>), dim3(wg), dim3(256), 0, s, L);
  int rc;
  if ((rc = (int)hipGetLastError())) return rc;
  const long nred = (long)g.cout * g.ks * g.ks * g.cin;
  // elements per block: >= ~512 blocks when possible; the rest of the block's threads split the splits
  int EB = 64;
  while (EB > 4 && (nred + EB - 1) / EB < 512) EB >>= 1;
  r.EB = EB;
  r.SG = 256 / EB;
  r.wblocks = (int)((nred + EB - 1) / EB);
  r.db = bias_col ? db : nullptr;
  const int bblocks = bias_col ? (g.cout + EB - 1) / EB : 0;
  if (t_wdefer.on && t_wdefer.m.n < CGL_WDEFER_MAX && (!db || bias_col || t_wdefer.m.nfin < CGL_WDEFER_FIN)) {
    CglWgradReduceMulti& m = t_wdefer.m;
    m.r[m.n] = r;
    m.begin[m.n + 1] = m.begin[m.n] + r.wblocks + bblocks;
    ++m.n;
    if (db && !bias_col) {   // the bias gradient's column-sum pass now, its finish with the reductions
      double* bp = (double*)(((uintptr_t)part + 255) & ~(uintptr_t)255);
      CglBnFinArgs f;
      if ((rc = col_sum_part(dY, (int64_t)g.n * g.ho * g.wo, g.cout, bp, db, s, f))) return rc;
      t_wdefer.add_fin(f);
    }
    return 0;
  }
  hipLaunchKernelGGL(cgl_conv_wgrad_reduce, dim3((unsigned)(r.wblocks + bblocks)), dim3(256), 0, s, r);
  if ((rc = (int)hipGetLastError())) return rc;
  if (db && !bias_col) {
    double* bp = (double*)(((uintptr_t)part + 255) & ~(uintptr_t)255);
    if ((rc = col_sum(dY, (int64_t)g.n * g.ho * g.wo, g.cout, bp, db, s))) return rc;
  }
  return 0;
}

}  // namespace

// ==========================================================================================
extern "C" {

int64_t cgl_conv3x3_workspace_bytes(int n, int h, int w, int cin, int cout, int stride, int up) {
  ConvGeom g;
  const int rc = conv_geom(n, h, w, cin, cout, stride, up, g);
  if (rc) return rc;
  return conv_ws_bytes(g);
}

int cgl_conv3x3_bias_by_colsum(int n, int h, int w, int cin, int cout, int stride, int up) {
  ConvGeom g;
  const int rc = conv_geom(n, h, w, cin, cout, stride, up, g);
  if (rc) return rc;
  if (c1_ok(g)) return 0;
  const WgradPlan pl = wgrad_plan(g, true);
  return (wgrad_bias_col(g, pl.P, pl.np) || !pow2_le256(cout)) ? 0 : 1;
}

int cgl_conv3x3_fwd(const float* X, const float* W, const float* bias, float* Y, int n, int h, int w, int cin,
                    int cout, int stride, int up, int act, float slope, const float* drop, void* ws, int64_t wsb,
                    void* stream) {
  CGL_BATCH_GUARD();
  ConvGeom g;
  const int rc = conv_geom(n, h, w, cin, cout, stride, up, g);
  if (rc) return rc;
  return conv_fwd_impl(g, X, W, bias, Y, act, slope, drop, ws, wsb, (hipStream_t)stream);
}

int cgl_conv3x3_bwd_data(const float* dY, const float* W, float* dX, int n, int h, int w, int cin, int cout,
                         int stride, int up, void* ws, int64_t wsb, void* stream) {
  CGL_BATCH_GUARD();
  ConvGeom g;
  const int rc = conv_geom(n, h, w, cin, cout, stride, up, g);
  if (rc) return rc;
  return conv_bwd_data_impl(g, dY, W, dX, ws, wsb, (hipStream_t)stream);
}

int cgl_conv3x3_bwd_weight(const float* dY, const float* X, float* dW, float* db, int n, int h, int w, int cin,
                           int cout, int stride, int up, void* ws, int64_t wsb, void* stream) {
  CGL_BATCH_GUARD();
  ConvGeom g;
  const int rc = conv_geom(n, h, w, cin, cout, stride, up, g);
  if (rc) return rc;
  return conv_bwd_weight_impl(g, dY, X, dW, db, ws, wsb, (hipStream_t)stream);
}

int cgl_conv3x3_bwd_weight_actdrop(const float* dY, const float* post, const float* drop, float slope, const float* X,
                                   float* dW, float* db, int n, int h, int w, int cin, int cout, int stride, int up,
                                   void* ws, int64_t wsb, void* stream) {
  CGL_BATCH_GUARD();
  ConvGeom g;
  const int rc = conv_geom(n, h, w, cin, cout, stride, up, g);
  if (rc) return rc;
  if (!c1_ok(g)) return CGL_E_ARG;     // the one-input-channel weight gradient only
  return conv_bwd_weight_impl(g, dY, X, dW, db, ws, wsb, (hipStream_t)stream, nullptr, post, drop, slope);
}

int cgl_conv3x3_bwd_weight_bnin(const float* dY, const float* X, float* dW, float* db, int n, int h, int w, int cin,
                                int cout, int stride, int up, const float* in_coef, int in_groups, int in_group,
                                int in_act, float in_slope, void* ws, int64_t wsb, void* stream) {
  CGL_BATCH_GUARD();
  ConvGeom g;
  const int rc = conv_geom(n, h, w, cin, cout, stride, up, g);
  if (rc) return rc;
  // in_group >= 0: every image is of that forward call; -1: n / in_groups images per call, stacked
  if (!in_coef || in_groups < 1 || in_group < -1 || in_group >= in_groups || (in_act != 0 && in_act != 1) ||
      (in_group < 0 && n % in_groups))
    return CGL_E_ARG;
  BnIn bi;
  bi.coef = in_coef;
  bi.groups = in_groups;
  bi.gimg = in_group >= 0 ? n : n / in_groups;
  bi.act = in_act;
  bi.slope = in_slope;
  bi.g0 = in_group >= 0 ? in_group : 0;
  return conv_bwd_weight_impl(g, dY, X, dW, db, ws, wsb, (hipStream_t)stream, &bi);
}

int64_t cgl_dense_workspace_bytes(int M, int K, int N) {
  ConvGeom g;
  const int rc = conv_geom(M, 1, 1, K, N, 1, 0, g, 1);
  if (rc) return rc;
  return conv_ws_bytes(g);
}

int cgl_dense_fwd(const float* X, const float* W, const float* b, float* Y, int M, int K, int N, int act, float slope,
                  void* ws, int64_t wsb, void* stream) {
  CGL_BATCH_GUARD();
  ConvGeom g;
  const int rc = conv_geom(M, 1, 1, K, N, 1, 0, g, 1);
  if (rc) return rc;
  return conv_fwd_impl(g, X, W, b, Y, act, slope, nullptr, ws, wsb, (hipStream_t)stream);
}

int cgl_dense_bwd_data(const float* dY, const float* W, float* dX, int M, int K, int N, void* ws, int64_t wsb,
                       void* stream) {
  CGL_BATCH_GUARD();
  ConvGeom g;
  const int rc = conv_geom(M, 1, 1, K, N, 1, 0, g, 1);
  if (rc) return rc;
  return conv_bwd_data_impl(g, dY, W, dX, ws, wsb, (hipStream_t)stream);
}

int cgl_dense_bwd_weight(const float* dY, const float* X, float* dW, float* db, int M, int K, int N, void* ws,
                         int64_t wsb, void* stream) {
  CGL_BATCH_GUARD();
  ConvGeom g;
  const int rc = conv_geom(M, 1, 1, K, N, 1, 0, g, 1);
  if (rc) return rc;
  // N = 1 (adv_layer): the one-launch kernel (CGL_DENSE1_WG=0: the implicit-GEMM weight gradient)
  static const int d1 = getenv("CGL_DENSE1_WG") ? atoi(getenv("CGL_DENSE1_WG")) : 1;
  if (d1 && N == 1 && dY && X && dW && (int64_t)M * K < ((int64_t)1 << 31)) {
    if (t_wdefer.on && t_wdefer.m.d1_blocks == 0) {   // rides in the deferred reductions' launch
      CglWgradReduceMulti& m = t_wdefer.m;
      m.d1_dy = dY; m.d1_x = X; m.d1_dw = dW; m.d1_db = db; m.d1_M = M; m.d1_K = K;
      m.d1_blocks = (K + 15) / 16 + 1;
      return CGL_OK;
    }
    hipLaunchKernelGGL(cgl_dense1_wgrad_k, dim3((K + 15) / 16 + 1), dim3(256), 0, (hipStream_t)stream, dY, X, dW, db,
                       M, K);
    return (int)hipGetLastError();
  }
  return conv_bwd_weight_impl(g, dY, X, dW, db, ws, wsb, (hipStream_t)stream);
}

int64_t cgl_conv_packed_floats(int h, int w, int cin, int cout, int stride, int up, int ks, int dir) {
  ConvGeom g;
  const int rc = conv_geom(1, h, w, cin, cout, stride, up, g, ks);
  if (rc) return rc;
  if (dir != 0 && dir != 1) return CGL_E_ARG;
  CglConvProb P[CGL_CONV_MAXP];
  const int np = dir ? bwd_probs(g, P) : fwd_probs(g, P);
  return pack_layout(P, np, nullptr);
}

int cgl_conv_wgrad_defer_begin(void) {
  if (t_wdefer.on) return CGL_E_STATE;
  t_wdefer = WgradDefer{};
  t_wdefer.on = true;
  return CGL_OK;
}

int cgl_conv_wgrad_defer_counters(int* counters, int n, int v, int* snap, int snap_index) {
  if (!t_wdefer.on || t_wdefer.m.cnt) return CGL_E_STATE;
  if (!counters || !snap || n < 1 || n > 64 || snap_index < 0 || snap_index >= n) return CGL_E_ARG;
  CglWgradReduceMulti& m = t_wdefer.m;
  m.cnt = counters; m.cnt_snap = snap; m.cnt_n = n; m.cnt_v = v; m.cnt_si = snap_index;
  return CGL_OK;
}

int cgl_conv_wgrad_defer_end(void* stream) {
  if (!t_wdefer.on) return CGL_E_STATE;
  t_wdefer.on = false;
  CglWgradReduceMulti& m = t_wdefer.m;
  if (!t_wdefer.has_c1) m.c1_blocks = 0;
  const int blocks = m.begin[m.n] + m.c1_blocks + m.fbeg[m.nfin] + m.d1_blocks + (m.cnt ? 1 : 0);
  if (blocks == 0) return CGL_OK;
  hipLaunchKernelGGL(cgl_conv_wgrad_reduce_multi, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, m);
  return (int)hipGetLastError();
}

// Launch batching (cgl_conv_batch_begin / _end): between the two calls, cgl_conv_pack_multi,
// cgl_dropout2d_masks(_dev), cgl_normal_fill_dev, cgl_sample_rows_dev and cgl_adv_loss (two at most) record their
// (validated) arguments instead of launching (one of each at most); _end launches them as one cgl_conv_begin_k.
// Every other launching entry point of the library returns CGL_E_STATE while a batch is open on the calling
// thread (CGL_BATCH_GUARD), so nothing can be launched ahead of the deferred calls on the stream.
namespace {
struct ConvBatch {
  bool on = false;
  hipStream_t s = nullptr;
  CglConvBeginArgs a{};
};
thread_local ConvBatch t_batch;
}  // namespace

}  // extern "C"
bool cgl_launch_batch_open() { return t_batch.on; }
extern "C" {

int cgl_conv_batch_begin(void* stream) {
  if (t_batch.on) return CGL_E_ARG;
  t_batch.on = true;
  t_batch.s = (hipStream_t)stream;
  std::memset(&t_batch.a, 0, sizeof(t_batch.a));
  return 0;
}

int cgl_conv_batch_end(void* stream) {
  if (!t_batch.on || (hipStream_t)stream != t_batch.s) return CGL_E_ARG;
  t_batch.on = false;
  const CglConvBeginArgs& a = t_batch.a;
  const int blk = a.pb + a.mb + a.nb + a.sb + a.lb;
  if (blk == 0) return 0;
  hipLaunchKernelGGL(cgl_conv_begin_k, dim3(blk), dim3(256), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

int cgl_conv_pack_multi(int njobs, const CglConvPackJob* jobs, void* stream) {
  if (njobs < 1 || !jobs) return CGL_E_ARG;
  CglPackMultiArgs a;
  std::memset(&a, 0, sizeof(a));
  int nj = 0, blk = 0;
  for (int i = 0; i < njobs; ++i) {
    const CglConvPackJob& J = jobs[i];
    ConvGeom g;
    int rc = conv_geom(1, J.h, J.w, J.cin, J.cout, J.stride, J.up, g, J.ks);
    if (rc) return rc;
    if (!J.W || !J.Wp || !al16(J.Wp) || (J.dir != 0 && J.dir != 1)) return CGL_E_ARG;
    CglConvProb P[CGL_CONV_MAXP];
    const int np = J.dir ? bwd_probs(g, P) : fwd_probs(g, P);
    pack_layout(P, np, J.Wp);
    for (int p = 0; p < np; ++p) {
      if (nj == CGL_PACKM_MAXJ) return CGL_E_SIZE;
      CglPackJobK& k = a.j[nj++];
      k.W = J.W;
      k.dst = const_cast<float*>(P[p].Wp);
      k.cout = g.cout; k.cin = g.cin; k.transpose = J.dir; k.ks = g.ks;
      k.N = P[p].N; k.Kp = P[p].Kp; k.Cg = P[p].Cin; k.Tx = P[p].Tx; k.T = P[p].Ty * P[p].Tx;
      k.tapm = 0;
      for (int t = 0; t < 4; ++t) k.tapm |= (P[p].ym[t] & 15) << (4 * t) | (P[p].xm[t] & 15) << (16 + 4 * t);
      k.blk_begin = blk;
      blk += (int)(((int64_t)P[p].N * P[p].Kp + 255) / 256);
    }
  }
  a.nj = nj;
  if (t_batch.on) {
    if (t_batch.a.pb || (hipStream_t)stream != t_batch.s) return CGL_E_ARG;
    t_batch.a.pack = a;
    t_batch.a.pb = blk;
    return 0;
  }
  hipLaunchKernelGGL(cgl_conv_pack_multi, dim3(blk), dim3(256), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

int cgl_conv3x3_fwd_packed(const float* X, const float* Wp, const float* bias, float* Y, int n, int h, int w, int cin,
                           int cout, int stride, int up, int act, float slope, const float* drop, void* ws,
                           int64_t wsb, void* stream) {
  CGL_BATCH_GUARD();
  ConvGeom g;
  const int rc = conv_geom(n, h, w, cin, cout, stride, up, g);
  if (rc) return rc;
  if (!Wp) return CGL_E_ARG;
  return conv_fwd_impl(g, X, nullptr, bias, Y, act, slope, drop, ws, wsb, (hipStream_t)stream, Wp);
}

int64_t cgl_conv3x3_stat_chunks(int n, int h, int w, int cin, int cout, int stride, int up, int groups) {
  ConvGeom g;
  const int rc = conv_geom(n, h, w, cin, cout, stride, up, g);
  if (rc) return rc;
  return (int64_t)stat_chunks_per_group(g, groups) * groups;
}

int cgl_conv3x3_fwd_packed_stats(const float* X, const float* Wp, const float* bias, float* Y, int n, int h, int w,
                                 int cin, int cout, int stride, int up, int act, float slope, const float* drop,
                                 int groups, double* part, const int* nvalid, void* ws, int64_t wsb, void* stream) {
  CGL_BATCH_GUARD();
  ConvGeom g;
  const int rc = conv_geom(n, h, w, cin, cout, stride, up, g);
  if (rc) return rc;
  if (!Wp || !part) return CGL_E_ARG;
  return conv_fwd_impl(g, X, nullptr, bias, Y, act, slope, drop, ws, wsb, (hipStream_t)stream, Wp, part, groups,
                       nullptr, nvalid);
}

int cgl_conv3x3_fwd_packed_bnin(const float* X, const float* Wp, const float* bias, float* Y, int n, int h, int w,
                                int cin, int cout, int stride, int up, int act, float slope, const float* drop,
                                int groups, double* part, const float* in_coef, int in_groups, int in_act,
                                float in_slope, const int* nvalid, void* ws, int64_t wsb, void* stream) {
  CGL_BATCH_GUARD();
  ConvGeom g;
  const int rc = conv_geom(n, h, w, cin, cout, stride, up, g);
  if (rc) return rc;
  if (!Wp || !in_coef || in_groups < 1 || n % in_groups) return CGL_E_ARG;
  BnIn bi;
  bi.coef = in_coef;
  bi.groups = in_groups;
  bi.gimg = n / in_groups;
  bi.act = in_act;
  bi.slope = in_slope;
  if (nvalid && !part) return CGL_E_ARG;
  return conv_fwd_impl(g, X, nullptr, bias, Y, act, slope, drop, ws, wsb, (hipStream_t)stream, Wp, part,
                       part ? groups : 1, &bi, nvalid);
}

int64_t cgl_conv3x3_bwd_stat_chunks(int n, int h, int w, int cin, int cout, int stride, int up, int groups) {
  ConvGeom g;
  const int rc = conv_geom(n, h, w, cin, cout, stride, up, g);
  if (rc) return rc;
  return (int64_t)stat_chunks_per_group(g, groups, 1) * groups;
}

int cgl_conv3x3_bwd_data_packed_stats(const float* dY, const float* Wp, float* dX, int n, int h, int w, int cin,
                                      int cout, int stride, int up, int groups, double* part, const float* bn_x,
                                      const float* bn_post, const float* bn_post_coef, int bn_post_coef_ld,
                                      const float* bn_mean, float slope, void* ws, int64_t wsb, void* stream) {
  CGL_BATCH_GUARD();
  ConvGeom g;
  const int rc = conv_geom(n, h, w, cin, cout, stride, up, g);
  if (rc) return rc;
  if (!Wp || !part || (bn_post_coef && (bn_post || groups != 1))) return CGL_E_ARG;
  StatBwd sb;
  sb.x = bn_x; sb.post = bn_post; sb.mean = bn_mean; sb.slope = slope;
  sb.psc = bn_post_coef; sb.psc_ld = bn_post_coef_ld;
  return conv_bwd_data_impl(g, dY, nullptr, dX, ws, wsb, (hipStream_t)stream, Wp, part, groups, &sb);
}

int cgl_conv3x3_bwd_data_stats(const float* dY, const float* W, float* dX, int n, int h, int w, int cin, int cout,
                               int stride, int up, int groups, double* part, const float* bn_x, const float* bn_post,
                               const float* bn_post_coef, int bn_post_coef_ld, const float* bn_mean, float slope,
                               void* ws, int64_t wsb, void* stream) {
  CGL_BATCH_GUARD();
  ConvGeom g;
  const int rc = conv_geom(n, h, w, cin, cout, stride, up, g);
  if (rc) return rc;
  // the vector one-output-channel input gradient (Conv2d(64, 1, 3, 1, 1)) only; partials per 128-row chunk
  if (!dY || !W || !dX || !part || !bn_x || !bn_mean || (bn_post_coef && (bn_post || groups != 1))) return CGL_E_ARG;
  if (g.cout != 1 || g.cin != 64 || g.ks != 3 || g.stride != 1 || g.up || groups < 1 || n % groups) return CGL_E_ARG;
  if (!al16(dX) || !al16(bn_x) || !al16(bn_mean) || (bn_post && !al16(bn_post)) || ((uintptr_t)part & 15))
    return CGL_E_ARG;
  if (bn_post_coef && (!al16(bn_post_coef) || bn_post_coef_ld % 4)) return CGL_E_ARG;
  const int64_t gr = (int64_t)(n / groups) * h * w;
  if (gr % (16 * CGL_BN1_PPT) || (int64_t)n * h * w >= (int64_t)1 << 30) return CGL_E_ARG;
  (void)ws; (void)wsb;
  const int npix = n * h * w;
  CglN1Stats st;
  st.X = bn_x; st.post = bn_post; st.psc = bn_post_coef; st.psc_ld = bn_post_coef_ld; st.mean = bn_mean;
  st.slope = slope; st.gr = (int)gr; st.part = part;
  hipLaunchKernelGGL((cgl_conv_bwd_n1<16, true>), dim3(npix / (16 * CGL_BN1_PPT)), dim3(256), 0, (hipStream_t)stream,
                     dY, W, dX, npix, g.h, g.w, st);
  return (int)hipGetLastError();
}

int cgl_conv3x3_bwd_data_packed(const float* dY, const float* W, const float* Wp, float* dX, int n, int h, int w,
                                int cin, int cout, int stride, int up, void* ws, int64_t wsb, void* stream) {
  CGL_BATCH_GUARD();
  ConvGeom g;
  const int rc = conv_geom(n, h, w, cin, cout, stride, up, g);
  if (rc) return rc;
  if (!Wp) return CGL_E_ARG;
  return conv_bwd_data_impl(g, dY, W, dX, ws, wsb, (hipStream_t)stream, Wp);
}

int cgl_dense_fwd_packed(const float* X, const float* Wp, const float* b, float* Y, int M, int K, int N, int act,
                         float slope, void* ws, int64_t wsb, void* stream) {
  CGL_BATCH_GUARD();
  ConvGeom g;
  const int rc = conv_geom(M, 1, 1, K, N, 1, 0, g, 1);
  if (rc) return rc;
  if (!Wp) return CGL_E_ARG;
  return conv_fwd_impl(g, X, nullptr, b, Y, act, slope, nullptr, ws, wsb, (hipStream_t)stream, Wp);
}

int cgl_dense_bwd_data_packed(const float* dY, const float* Wp, float* dX, int M, int K, int N, void* ws, int64_t wsb,
                              void* stream) {
  CGL_BATCH_GUARD();
  ConvGeom g;
  const int rc = conv_geom(M, 1, 1, K, N, 1, 0, g, 1);
  if (rc) return rc;
  if (!Wp) return CGL_E_ARG;
  return conv_bwd_data_impl(g, dY, nullptr, dX, ws, wsb, (hipStream_t)stream, Wp);
}

int64_t cgl_bn2d_workspace_bytes(int n, int hw, int C, int groups) {
  if (n < 1 || hw < 1 || C < 1 || groups < 1 || n % groups) return CGL_E_ARG;
  const int64_t gr = (int64_t)(n / groups) * hw;
  const int R = chan_chunk(gr);
  const int64_t nch = (int64_t)n * hw / R;
  return al256(nch * C * 16) + 4 * al256((int64_t)groups * C * 4) + 256;
}

int cgl_bn2d_fwd(const float* X, int n, int hw, int C, int groups, const float* gamma, const float* beta, double eps,
                 double momentum, float* running_mean, float* running_var, int train, int act, float slope, float* Y,
                 float* save_mean, float* save_invstd, const int* nvalid, void* ws, int64_t wsb, void* stream) {
  CGL_BATCH_GUARD();
  if (!X || !Y || !gamma || !beta || !ws || !al16(ws) || !al16(X) || !al16(Y)) return CGL_E_ARG;
  if (n < 1 || hw < 1 || C % 4 != 0 || !pow2_le256(C) || groups < 1 || n % groups || (act != 0 && act != 1))
    return CGL_E_ARG;
  if ((running_mean == nullptr) != (running_var == nullptr)) return CGL_E_ARG;
  if ((save_mean == nullptr) != (save_invstd == nullptr)) return CGL_E_ARG;
  if (!train && !running_mean) return CGL_E_ARG;
  const int64_t gr = (int64_t)(n / groups) * hw;
  if (train && gr < 2) return CGL_E_ARG;   // torch: "Expected more than 1 value per channel when training"
  if (wsb < cgl_bn2d_workspace_bytes(n, hw, C, groups)) return CGL_E_SIZE;
  hipStream_t s = (hipStream_t)stream;
  const int R = chan_chunk(gr);
  const int64_t rows = (int64_t)n * hw;
  const int nch = (int)(rows / R);
  double* part = (double*)ws;
  float* coef = (float*)((char*)ws + al256((int64_t)nch * C * 16));
  float* c0 = coef;
  float* c1 = coef + al256((int64_t)groups * C * 4) / 4;
  if (train) {
    CglChanArgs a;
    std::memset(&a, 0, sizeof(a));
    a.X = X; a.rows = (int)rows; a.C = C; a.R = R; a.mode = 0; a.gr = (int)gr; a.part = part;
    a.nv = nvalid; a.hw = hw;
    launch_chan_reduce(a, nch, s);
  }
  CglBnFinArgs f;
  std::memset(&f, 0, sizeof(f));
  f.part = part; f.C = C; f.groups = groups; f.chunks_per_group = (int)(gr / R); f.R = R; f.gr = (int)gr;
  f.nv = train ? nvalid : nullptr; f.hw = hw;
  f.mode = 0; f.train = train; f.gamma = gamma; f.beta = beta; f.eps = eps; f.momentum = momentum;
  f.run_mean = running_mean; f.run_var = running_var; f.save_mean = save_mean; f.save_invstd = save_invstd;
  f.coef0 = c0; f.coef1 = c1;
  f.nocache = fin_nocache();
  hipLaunchKernelGGL(cgl_bn_finalize, dim3(C), dim3(256), 0, s, f);
  CglEltArgs e;
  std::memset(&e, 0, sizeof(e));
  e.mode = 0; e.rows = (int)rows; e.C = C; e.gr = (int)gr; e.hw = hw; e.act = act; e.slope = slope;
  e.X = X; e.coef0 = c0; e.coef1 = c1; e.out = Y;
  const long n4 = rows * C / 4;
  hipLaunchKernelGGL(cgl_eltwise, dim3((unsigned)std::min<long>((n4 + 255) / 256, 8192)), dim3(256), 0, s, e);
  return (int)hipGetLastError();
}

int64_t cgl_bn2d_stats_scratch_bytes(int C, int groups) {
  if (C < 1 || groups < 1) return CGL_E_ARG;
  return al256((int64_t)C * 4) + (int64_t)C * groups * CGL_FIN_MAXS * 16;
}

int cgl_bn2d_fwd_stats(const double* part, int R, const float* X, int n, int hw, int C, int groups, const float* gamma,
                       const float* beta, double eps, double momentum, float* running_mean, float* running_var,
                       int act, float slope, float* Y, float* save_mean, float* save_invstd, void* scratch,
                       const int* nvalid, void* ws, int64_t wsb, void* stream) {
  CGL_BATCH_GUARD();
  return cgl_bn2d_fwd_stats_coef(part, R, X, n, hw, C, groups, gamma, beta, eps, momentum, running_mean, running_var,
                                 act, slope, Y, save_mean, save_invstd, scratch, nullptr, 0, nvalid, ws, wsb, stream);
}

int cgl_bn2d_fwd_stats_coef(const double* part, int R, const float* X, int n, int hw, int C, int groups,
                            const float* gamma, const float* beta, double eps, double momentum, float* running_mean,
                            float* running_var, int act, float slope, float* Y, float* save_mean, float* save_invstd,
                            void* scratch, float* coef, int apply_img0, const int* nvalid, void* ws, int64_t wsb,
                            void* stream) {
  CGL_BATCH_GUARD();
  if (!part || !X || !Y || !gamma || !beta || !ws || !al16(ws) || !al16(X) || !al16(Y)) return CGL_E_ARG;
  if ((coef && !al16(coef)) || apply_img0 < 0 || apply_img0 > n) return CGL_E_ARG;
  if (n < 1 || hw < 1 || C % 4 != 0 || !pow2_le256(C) || groups < 1 || n % groups || (act != 0 && act != 1))
    return CGL_E_ARG;
  if ((running_mean == nullptr) != (running_var == nullptr)) return CGL_E_ARG;
  if ((save_mean == nullptr) != (save_invstd == nullptr)) return CGL_E_ARG;
  const int64_t gr = (int64_t)(n / groups) * hw;
  if (R < 1 || gr % R || gr < 2) return CGL_E_ARG;
  if (wsb < cgl_bn2d_workspace_bytes(n, hw, C, groups)) return CGL_E_SIZE;
  hipStream_t s = (hipStream_t)stream;
  const int64_t rows = (int64_t)n * hw;
  const int R0 = chan_chunk(gr);
  float* cbuf = coef ? coef : (float*)((char*)ws + al256((rows / R0) * C * 16));
  float* c0 = cbuf;
  float* c1 = coef ? coef + (int64_t)groups * C : cbuf + al256((int64_t)groups * C * 4) / 4;
  CglBnFinArgs f;
  std::memset(&f, 0, sizeof(f));
  f.part = part; f.C = C; f.groups = groups; f.chunks_per_group = (int)(gr / R); f.R = R; f.gr = (int)gr;
  f.mode = 0; f.train = 1; f.gamma = gamma; f.beta = beta; f.eps = eps; f.momentum = momentum;
  f.nv = nvalid; f.hw = hw;
  f.run_mean = running_mean; f.run_var = running_var; f.save_mean = save_mean; f.save_invstd = save_invstd;
  f.coef0 = c0; f.coef1 = c1;
  const int cpg = (int)(gr / R);
  if (scratch && cpg > 1024) {   // many chunks: slices of <= 512 per block, merged by the last block
    if ((uintptr_t)scratch & 255) return CGL_E_ARG;
    CglBnFinSliced a;
    std::memset(&a, 0, sizeof(a));
    a.f = f;
    a.L = 512;
    a.S = (cpg + a.L - 1) / a.L;
    if (a.S > CGL_FIN_MAXS) a.L = (cpg + CGL_FIN_MAXS - 1) / CGL_FIN_MAXS, a.S = (cpg + a.L - 1) / a.L;
    a.ctr = (unsigned int*)scratch;
    a.sl = (double*)((char*)scratch + al256((int64_t)C * 4));
    hipLaunchKernelGGL(cgl_bn_finalize_sliced, dim3(a.S, C), dim3(256), 0, s, a);
  } else {
    f.nocache = fin_nocache();
  hipLaunchKernelGGL(cgl_bn_finalize, dim3(C), dim3(256), 0, s, f);
  }
  // apply to images [apply_img0, n) only (a consumer folds the rest into its operand load from `coef`)
  const int64_t row0 = (int64_t)apply_img0 * hw, arows = rows - row0;
  if (arows <= 0) return (int)hipGetLastError();
  CglEltArgs e;
  std::memset(&e, 0, sizeof(e));
  e.mode = 0; e.rows = (int)arows; e.C = C; e.gr = (int)gr; e.hw = hw; e.act = act; e.slope = slope;
  e.row0 = (int)row0;
  e.X = X + row0 * C; e.coef0 = c0; e.coef1 = c1; e.out = Y + row0 * C;
  const long n4 = arows * C / 4;
  hipLaunchKernelGGL(cgl_eltwise, dim3((unsigned)std::min<long>((n4 + 255) / 256, 8192)), dim3(256), 0, s, e);
  return (int)hipGetLastError();
}

int cgl_bn2d_bwd_stats(const double* part, int R, const float* dY, const float* post, const float* X, int n, int hw,
                       int C, int groups, const float* save_mean, const float* save_invstd, const float* gamma,
                       float slope, const float* post_out, const float* drop, float* dX, float* dgamma, float* dbeta,
                       const float* post_coef, int post_coef_ld, const int* nvalid, double* colsum_part, void* ws,
                       int64_t wsb, void* stream) {
  CGL_BATCH_GUARD();
  if (post_coef && (post || groups != 1 || !al16(post_coef) || post_coef_ld % 4)) return CGL_E_ARG;
  if (colsum_part && (((uintptr_t)colsum_part & 15) || C % 4 || 256 % (C / 4) || ((int64_t)n * hw) % 256))
    return CGL_E_ARG;
  if (!part || !dY || !X || !save_mean || !save_invstd || !gamma || !dX || !ws || !al16(ws)) return CGL_E_ARG;
  if (!al16(dY) || !al16(X) || !al16(dX) || (post && !al16(post)) || (post_out && !al16(post_out))) return CGL_E_ARG;
  if (!al16(save_mean) || !al16(save_invstd) || !al16(gamma) || (drop && !al16(drop))) return CGL_E_ARG;
  if (n < 1 || hw < 1 || C % 4 != 0 || !pow2_le256(C) || groups < 1 || n % groups) return CGL_E_ARG;
  const int64_t gr = (int64_t)(n / groups) * hw;
  if (R < 1 || gr % R) return CGL_E_ARG;
  if (wsb < cgl_bn2d_workspace_bytes(n, hw, C, groups)) return CGL_E_SIZE;
  hipStream_t s = (hipStream_t)stream;
  const int64_t rows = (int64_t)n * hw;
  const int R0 = chan_chunk(gr);
  float* coef = (float*)((char*)ws + al256((rows / R0) * C * 16));
  float* c0 = coef;
  float* c1 = coef + al256((int64_t)groups * C * 4) / 4;
  CglBnFinArgs f;
  std::memset(&f, 0, sizeof(f));
  f.part = part; f.C = C; f.groups = groups; f.chunks_per_group = (int)(gr / R); f.R = R; f.gr = (int)gr;
  f.mode = 1; f.gamma = gamma; f.save_invstd = const_cast<float*>(save_invstd); f.coef0 = c0; f.coef1 = c1;
  f.dgamma = dgamma; f.dbeta = dbeta;
  f.nv = nvalid; f.hw = hw;
  f.nocache = fin_nocache();
  hipLaunchKernelGGL(cgl_bn_finalize, dim3(C), dim3(256), 0, s, f);
  CglEltArgs e;
  std::memset(&e, 0, sizeof(e));
  e.mode = 1; e.rows = (int)rows; e.C = C; e.gr = (int)gr; e.hw = hw; e.slope = slope;
  e.X = X; e.dY = dY; e.post = post; e.coef0 = c0; e.coef1 = c1; e.mean = save_mean; e.invstd = save_invstd;
  e.gamma = gamma; e.post_out = post_out; e.drop = drop; e.out = dX; e.nv = nvalid;
  e.psc = post_coef; e.psc_ld = post_coef_ld;
  const long n4 = rows * C / 4;
  if (colsum_part) {   // + the output's column sums per 256-row chunk (a bias gradient's col_sum partials)
    hipLaunchKernelGGL(cgl_bnb_apply_colsum<CGL_BNB_NB>, dim3((unsigned)(rows / 256)), dim3(256), 0, s, e, colsum_part);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(cgl_eltwise, dim3((unsigned)std::min<long>((n4 + 255) / 256, 8192)), dim3(256), 0, s, e);
  return (int)hipGetLastError();
}

int cgl_bn2d_bwd(const float* dY, const float* post, const float* X, int n, int hw, int C, int groups,
                 const float* save_mean, const float* save_invstd, const float* gamma, float slope,
                 const float* post_out, const float* drop, float* dX, float* dgamma, float* dbeta,
                 const float* post_coef, int post_coef_ld, const int* nvalid, void* ws, int64_t wsb, void* stream) {
  CGL_BATCH_GUARD();
  if (post_coef && (post || groups != 1 || !al16(post_coef) || post_coef_ld % 4)) return CGL_E_ARG;
  if (!dY || !X || !save_mean || !save_invstd || !gamma || !dX || !ws || !al16(ws)) return CGL_E_ARG;
  if (!al16(dY) || !al16(X) || !al16(dX) || (post && !al16(post)) || (post_out && !al16(post_out))) return CGL_E_ARG;
  if (!al16(save_mean) || !al16(save_invstd) || !al16(gamma) || (drop && !al16(drop))) return CGL_E_ARG;
  if (n < 1 || hw < 1 || C % 4 != 0 || !pow2_le256(C) || groups < 1 || n % groups) return CGL_E_ARG;
  if (wsb < cgl_bn2d_workspace_bytes(n, hw, C, groups)) return CGL_E_SIZE;
  hipStream_t s = (hipStream_t)stream;
  const int64_t gr = (int64_t)(n / groups) * hw;
  const int R = chan_chunk(gr);
  const int64_t rows = (int64_t)n * hw;
  const int nch = (int)(rows / R);
  double* part = (double*)ws;
  float* coef = (float*)((char*)ws + al256((int64_t)nch * C * 16));
  float* c0 = coef;
  float* c1 = coef + al256((int64_t)groups * C * 4) / 4;
  CglChanArgs a;
  std::memset(&a, 0, sizeof(a));
  a.X = X; a.rows = (int)rows; a.C = C; a.R = R; a.mode = 1; a.gr = (int)gr; a.part = part;
  a.dY = dY; a.post = post; a.slope = slope; a.mean = save_mean;
  a.psc = post_coef; a.psc_ld = post_coef_ld;
  launch_chan_reduce(a, nch, s);
  CglBnFinArgs f;
  std::memset(&f, 0, sizeof(f));
  f.part = part; f.C = C; f.groups = groups; f.chunks_per_group = (int)(gr / R); f.R = R; f.gr = (int)gr;
  f.mode = 1; f.gamma = gamma; f.save_invstd = const_cast<float*>(save_invstd); f.coef0 = c0; f.coef1 = c1;
  f.dgamma = dgamma; f.dbeta = dbeta;
  f.nv = nvalid; f.hw = hw;
  f.nocache = fin_nocache();
  hipLaunchKernelGGL(cgl_bn_finalize, dim3(C), dim3(256), 0, s, f);
  CglEltArgs e;
  std::memset(&e, 0, sizeof(e));
  e.mode = 1; e.rows = (int)rows; e.C = C; e.gr = (int)gr; e.hw = hw; e.slope = slope;
  e.X = X; e.dY = dY; e.post = post; e.coef0 = c0; e.coef1 = c1; e.mean = save_mean; e.invstd = save_invstd;
  e.gamma = gamma; e.post_out = post_out; e.drop = drop; e.out = dX; e.nv = nvalid;
  e.psc = post_coef; e.psc_ld = post_coef_ld;
  const long n4 = rows * C / 4;
  hipLaunchKernelGGL(cgl_eltwise, dim3((unsigned)std::min<long>((n4 + 255) / 256, 8192)), dim3(256), 0, s, e);
  return (int)hipGetLastError();
}

int cgl_act_drop_bwd(const float* dY, const float* post, const float* drop, int n, int hw, int C, float slope,
                     int tanh_y, float* dX, void* stream) {
  CGL_BATCH_GUARD();
  if (!dY || !dX || n < 1 || hw < 1 || C < 1) return CGL_E_ARG;
  if (tanh_y && !post) return CGL_E_ARG;
  hipStream_t s = (hipStream_t)stream;
  CglEltArgs e;
  std::memset(&e, 0, sizeof(e));
  e.mode = tanh_y ? 3 : 2;
  e.rows = n * hw; e.C = C; e.gr = n * hw; e.hw = hw; e.slope = slope;
  e.dY = dY; e.out = dX;
  if (tanh_y) e.X = post;
  else e.post_out = post;
  e.drop = drop;
  const long tot = (long)n * hw * C;
  const bool v4 = C % 4 == 0 && al16(dY) && al16(dX) && (!post || al16(post)) && (!drop || al16(drop));
  if (v4)
    hipLaunchKernelGGL(cgl_eltwise, dim3((unsigned)std::min<long>((tot / 4 + 255) / 256, 8192)), dim3(256), 0, s, e);
  else
    hipLaunchKernelGGL(cgl_eltwise1, dim3((unsigned)std::min<long>((tot + 255) / 256, 8192)), dim3(256), 0, s, e);
  return (int)hipGetLastError();
}

int cgl_act_drop_bwd_colsum(const float* dY, const float* post, const float* drop, int n, int hw, int C, float slope,
                            int tanh_y, float* dX, double* part, void* stream) {
  CGL_BATCH_GUARD();
  const long tot = (long)n * hw * C;
  if (!dY || !dX || !part || n < 1 || hw < 1 || C != 1 || tot > 8192L * 256 || ((uintptr_t)part & 15)) return CGL_E_ARG;
  if (tanh_y && !post) return CGL_E_ARG;
  CglEltArgs e;
  std::memset(&e, 0, sizeof(e));
  e.mode = tanh_y ? 3 : 2;
  e.rows = n * hw; e.C = C; e.gr = n * hw; e.hw = hw; e.slope = slope;
  e.dY = dY; e.out = dX;
  if (tanh_y) e.X = post;
  else e.post_out = post;
  e.drop = drop;
  e.colsum = part;
  hipLaunchKernelGGL(cgl_eltwise1, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, (hipStream_t)stream, e);
  return (int)hipGetLastError();
}

int cgl_colsum_finalize(const double* part, int nch, int C, float* out, void* stream) {
  CGL_BATCH_GUARD();
  if (!part || !out || nch < 1 || C < 1) return CGL_E_ARG;
  CglBnFinArgs f;
  std::memset(&f, 0, sizeof(f));
  f.part = part; f.C = C; f.groups = 1; f.chunks_per_group = nch; f.mode = 2; f.dgamma = out;
  f.nocache = fin_nocache();
  if (t_wdefer.on && t_wdefer.add_fin(f)) return CGL_OK;   // rides in the deferred reductions' launch
  hipLaunchKernelGGL(cgl_bn_finalize, dim3(C), dim3(256), 0, (hipStream_t)stream, f);
  return (int)hipGetLastError();
}

int cgl_dropout2d_mask(float* mask, int n, int C, double p, unsigned long long seed, unsigned long long counter,
                       void* stream) {
  CGL_BATCH_GUARD();
  if (!mask || n < 1 || C < 1 || !(p >= 0.0 && p < 1.0)) return CGL_E_ARG;
  const long tot = (long)n * C;
  const float keep = (float)(1.0 - p);
  const float scale = 1.0f / keep;
  hipLaunchKernelGGL(cgl_dropout_mask_k, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, (hipStream_t)stream, mask,
                     tot, keep, scale, seed, counter);
  return (int)hipGetLastError();
}

static int dropout2d_masks_impl(int nm, float* const* masks, const int* n, const int* C, double p,
                                unsigned long long seed, const unsigned long long* counters, const int* round_dev,
                                unsigned long long round_stride, void* stream) {
  if (nm < 1 || nm > CGL_MASKS_MAX || !masks || !n || !C || !counters || !(p >= 0.0 && p < 1.0)) return CGL_E_ARG;
  CglMasksArgs a;
  std::memset(&a, 0, sizeof(a));
  a.nm = nm;
  a.keep = (float)(1.0 - p);
  a.scale = 1.0f / a.keep;
  a.seed = seed;
  int blk = 0;
  for (int j = 0; j < nm; ++j) {
    if (!masks[j] || n[j] < 1 || C[j] < 1) return CGL_E_ARG;
    a.mask[j] = masks[j];
    a.n[j] = (long)n[j] * C[j];
    a.ctr[j] = counters[j];
    a.blk_begin[j] = blk;
    blk += (int)((a.n[j] + 255) / 256);
  }
  a.rdev = round_dev;
  a.rstride = round_stride;
  if (t_batch.on) {
    if (t_batch.a.mb || (hipStream_t)stream != t_batch.s) return CGL_E_ARG;
    t_batch.a.masks = a;
    t_batch.a.mb = blk;
    return 0;
  }
  hipLaunchKernelGGL(cgl_dropout_masks_k, dim3(blk), dim3(256), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

int cgl_dropout2d_masks(int nm, float* const* masks, const int* n, const int* C, double p, unsigned long long seed,
                        const unsigned long long* counters, void* stream) {
  return dropout2d_masks_impl(nm, masks, n, C, p, seed, counters, nullptr, 0, stream);
}

int cgl_nchw_to_nhwc(const float* X, float* Y, int n, int c, int hw, void* stream) {
  CGL_BATCH_GUARD();
  if (!X || !Y || n < 1 || c < 1 || hw < 1) return CGL_E_ARG;
  hipLaunchKernelGGL(cgl_transpose_k, dim3((hw + 31) / 32, (c + 31) / 32, n), dim3(256), 0, (hipStream_t)stream, X, Y,
                     c, hw);
  return (int)hipGetLastError();
}

int cgl_dense1_fwd_nhwc(const float* X, const float* W, const float* b, float* Y, float* flat, int n, int c, int hw,
                        void* stream) {
  CGL_BATCH_GUARD();
  const long per = (long)c * hw;
  if (!X || !W || !Y || n < 1 || c < 1 || hw < 1 || per % 256 || per > 1024 || (long)n * per >= (1L << 31) || !al16(W) ||
      (flat && !al16(flat)))
    return CGL_E_ARG;
  hipLaunchKernelGGL(cgl_dense1_fwd_nhwc_k, dim3((n + 3) / 4), dim3(256), 0, (hipStream_t)stream, X, W, b, Y, flat, n, c,
                     hw);
  return (int)hipGetLastError();
}

int cgl_dense1_bwd_data_nhwc(const float* dY, const float* W, float* dX, int n, int c, int hw, void* stream) {
  CGL_BATCH_GUARD();
  if (!dY || !W || !dX || n < 1 || c < 4 || (c & 3) || hw < 1 || (long)n * c * hw >= (1L << 31) || !al16(dX))
    return CGL_E_ARG;   // (the kernel stores float4 into dX)
  const long q = (long)n * c * hw / 4;
  const int grid = (int)std::min<long>((q + 255) / 256, 8192);
  hipLaunchKernelGGL(cgl_dense1_bwd_nhwc_k, dim3(grid), dim3(256), 0, (hipStream_t)stream, dY, W, dX, n, c, hw);
  return (int)hipGetLastError();
}

int cgl_dense1_head_nhwc(const float* X, const float* W, const float* b, float* Y, float* flat, float* dY, float* dX,
                         int n, int c, int hw, int loss, int n0, int target0, double weight0, float* loss_out0,
                         const int* nvalid0, int target1, double weight1, float* loss_out1, const float* in_coef,
                         int in_groups, float* scratch, void* stream) {
  CGL_BATCH_GUARD();
  const long per = (long)c * hw;
  if (in_coef && (in_groups < 1 || n % in_groups)) return CGL_E_ARG;
  if (!X || !W || !Y || !dY || !dX || !scratch || n < 1 || c < 4 || (c & 3) || hw < 1 || per % 256 || per > 1024 ||
      (long)n * per >= (1L << 31) || !al16(W) || !al16(dX) || (flat && !al16(flat)) || loss < 1 || loss > 3 ||
      n0 < 1 || n0 > n || (target0 != 0 && target0 != 1) || (n0 < n && target1 != 0 && target1 != 1))
    return CGL_E_ARG;
  CglDHeadArgs a;
  std::memset(&a, 0, sizeof(a));
  a.X = X; a.W = W; a.b = b; a.Y = Y; a.flat = flat; a.dY = dY; a.dX = dX;
  a.n = n; a.C = c; a.hw = hw; a.loss = loss; a.ncalls = n0 < n ? 2 : 1;
  a.call[0] = CglHeadCall{0, n0, target0, (float)weight0, loss_out0, nvalid0};
  a.call[1] = CglHeadCall{n0, n - n0, target1, (float)weight1, loss_out1, nullptr};
  a.ticket = (unsigned int*)scratch;
  a.lrow = scratch + 16;
  a.coef = in_coef;
  a.groups = in_coef ? in_groups : 1;
  hipLaunchKernelGGL(cgl_dense1_head_k, dim3((n + 3) / 4), dim3(256), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

int cgl_nhwc_to_nchw(const float* X, float* Y, int n, int c, int hw, void* stream) {
  CGL_BATCH_GUARD();
  if (!X || !Y || n < 1 || c < 1 || hw < 1) return CGL_E_ARG;
  hipLaunchKernelGGL(cgl_transpose_k, dim3((c + 31) / 32, (hw + 31) / 32, n), dim3(256), 0, (hipStream_t)stream, X, Y,
                     hw, c);
  return (int)hipGetLastError();
}

int cgl_adv_loss(const float* x, int M, int C, int loss, int target, double weight, float* loss_out, float* grad,
                 const int* nvalid, void* stream) {
  if (!x || M < 1 || loss < 0 || loss > 3 || (target != 0 && target != 1)) return CGL_E_ARG;
  if ((loss == 0) != (C == 2) || (loss != 0 && C != 1)) return CGL_E_ARG;
  if (t_batch.on) {
    if (t_batch.a.lb >= 2 || (hipStream_t)stream != t_batch.s) return CGL_E_ARG;
    CglAdvArgs& q = t_batch.a.adv[t_batch.a.lb++];
    q.x = x; q.Mall = M; q.C = C; q.loss = loss; q.target = target; q.weight = (float)weight; q.loss_out = loss_out;
    q.grad = grad; q.nv = nvalid;
    return 0;
  }
  hipLaunchKernelGGL(cgl_adv_loss_k, dim3(1), dim3(256), 0, (hipStream_t)stream, x, M, C, loss, target,
                     (float)weight, loss_out, grad, nvalid);
  return (int)hipGetLastError();
}

int cgl_weights_scale(int weighting, int n, int rank, float lam, const float* beta_host, const float* losses,
                      float* x, int64_t nx, float* alpha_out, void* stream) {
  CGL_BATCH_GUARD();
  if (weighting < 0 || weighting > 4 || n < 1 || n > CGL_MAX_WORKERS || rank < 0 || rank >= n || !beta_host ||
      !losses || (nx > 0 && !x) || nx < 0)
    return CGL_E_ARG;
  CglWeightsArgs a;
  std::memset(&a, 0, sizeof(a));
  a.mode = weighting; a.n = n; a.rank = rank; a.lam = lam;
  for (int q = 0; q < n; ++q) a.beta[q] = beta_host[q];
  a.losses = losses; a.x = x; a.nx = (long)nx; a.alpha_out = alpha_out;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((nx + 255) / 256, 1024));
  hipLaunchKernelGGL(cgl_weights_scale_k, dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

int cgl_gather_rows(const float* src, const int* idx, int64_t row0, int nrows, int row_floats, float* dst,
                    void* stream) {
  CGL_BATCH_GUARD();
  if (!src || !dst || nrows < 0 || row_floats < 1 || row0 < 0) return CGL_E_ARG;
  if (nrows == 0) return 0;
  const long n = (long)nrows * row_floats;
  hipLaunchKernelGGL(cgl_gather_rows_k, dim3((unsigned)std::min<long>((n + 255) / 256, 8192)), dim3(256), 0,
                     (hipStream_t)stream, src, idx, (long)row0, nrows, row_floats, dst);
  return (int)hipGetLastError();
}

static int adam_multi_impl(int nt, float* const* p, const float* const* g, float* const* m, float* const* v,
                           const int64_t* n, int step, const int* step_dev, double lr, double beta1, double beta2,
                           double eps, void* stream) {
  if (nt < 1 || nt > CGL_ADAM_MAXT || !p || !g || !m || !v || !n) return CGL_E_ARG;
  CglAdamMulti a;
  std::memset(&a, 0, sizeof(a));
  a.nt = nt;
  int blk = 0;
  for (int i = 0; i < nt; ++i) {
    if (!p[i] || !g[i] || !m[i] || !v[i] || n[i] < 0) return CGL_E_ARG;
    a.p[i] = p[i]; a.g[i] = g[i]; a.m[i] = m[i]; a.v[i] = v[i]; a.n[i] = (long)n[i];
    a.blk[i] = blk;
    blk += (int)((n[i] + 255) / 256);
  }
  a.blk[nt] = blk;
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  a.step_size = (float)(lr / bc1);
  a.bc2sqrt = (float)std::pow(bc2, 0.5);
  a.b2 = (float)beta2;
  a.w1 = (float)(1.0 - beta1);
  a.w2 = (float)(1.0 - beta2);
  a.eps = (float)eps;
  a.step_dev = step_dev;
  a.lr = lr;
  a.beta1 = beta1;
  a.beta2 = beta2;
  if (blk == 0) return 0;
  hipLaunchKernelGGL(cgl_adam_multi_k, dim3(blk), dim3(256), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

int cgl_adam_multi(int nt, float* const* p, const float* const* g, float* const* m, float* const* v,
                   const int64_t* n, int step, double lr, double beta1, double beta2, double eps, void* stream) {
  CGL_BATCH_GUARD();
  if (step < 1) return CGL_E_ARG;
  return adam_multi_impl(nt, p, g, m, v, n, step, nullptr, lr, beta1, beta2, eps, stream);
}

int cgl_adam_multi_dev(int nt, float* const* p, const float* const* g, float* const* m, float* const* v,
                       const int64_t* n, const int* step_dev, double lr, double beta1, double beta2, double eps,
                       void* stream) {
  CGL_BATCH_GUARD();
  if (!step_dev) return CGL_E_ARG;
  return adam_multi_impl(nt, p, g, m, v, n, 1, step_dev, lr, beta1, beta2, eps, stream);
}

int cgl_normal_fill_dev(float* out, int64_t n, unsigned long long seed, const int* round_dev, int stream_id,
                        void* stream) {
  if (!out || n < 0 || !round_dev) return CGL_E_ARG;
  if (n == 0) return 0;
  if (t_batch.on) {
    if (t_batch.a.nb || (hipStream_t)stream != t_batch.s) return CGL_E_ARG;
    CglConvBeginArgs& b = t_batch.a;
    b.n_out = out; b.n_n = (long)n; b.n_seed = seed; b.n_round = round_dev; b.n_sid = stream_id;
    b.nb = (int)((n / 4 + 255) / 256);
    return 0;
  }
  hipLaunchKernelGGL(cgl_normal_dev_k, dim3((unsigned)((n / 4 + 255) / 256)), dim3(256), 0, (hipStream_t)stream, out,
                     (long)n, seed, round_dev, stream_id);
  return (int)hipGetLastError();
}

int cgl_dropout2d_masks_dev(int nm, float* const* masks, const int* n, const int* C, double p,
                            unsigned long long seed, const unsigned long long* counters, const int* round_dev,
                            unsigned long long round_stride, void* stream) {
  if (!round_dev) return CGL_E_ARG;
  return dropout2d_masks_impl(nm, masks, n, C, p, seed, counters, round_dev, round_stride, stream);
}

int cgl_sample_rows_dev(const float* src, int n_src, int nrows, int row_floats, unsigned long long seed,
                        const int* round_dev, float* dst, int* nv_out, void* stream) {
  if (!src || !dst || !round_dev || nrows < 1 || n_src < 1 || (!nv_out && n_src < nrows) || row_floats < 4 ||
      row_floats % 4 || ((uintptr_t)src & 15) || ((uintptr_t)dst & 15))
    return CGL_E_ARG;
  if (t_batch.on) {
    if (t_batch.a.sb || (hipStream_t)stream != t_batch.s) return CGL_E_ARG;
    CglConvBeginArgs& b = t_batch.a;
    b.s_src = src; b.s_nsrc = n_src; b.s_nrows = nrows; b.s_rowf = row_floats; b.s_seed = seed; b.s_round = round_dev;
    b.s_dst = dst; b.s_nv = nv_out;
    b.sb = nrows;
    return 0;
  }
  hipLaunchKernelGGL(cgl_sample_rows_k, dim3(nrows), dim3(256), 0, (hipStream_t)stream, src, n_src, nrows, row_floats,
                     seed, round_dev, dst, nv_out);
  return (int)hipGetLastError();
}

int cgl_counters_add(int* p, int n, int v, void* stream) {
  CGL_BATCH_GUARD();
  if (!p || n < 1 || n > 64) return CGL_E_ARG;
  hipLaunchKernelGGL(cgl_counters_add_k, dim3(1), dim3(64), 0, (hipStream_t)stream, p, n, v);
  return (int)hipGetLastError();
}

}  // extern "C"
