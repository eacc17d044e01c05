// fp32 MFMA GEMM for the MLP GAN step (gfx950, v_mfma_f32_32x32x2_f32).
//
// Replaces the reference's implicit cuBLAS addmm / mm calls of nn.Linear forward and
// autograd backward (model/mnist_model.py:11,22,77,79,81).
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
//  * prologue fusion: the A operand rows can be gathered through an index list (the sampled
//    real batch) from two sources (real rows, then generated rows) and written out once;
//  * epilogue fusion: bias, LeakyReLU / Tanh, LeakyReLU' mask, Tanh' (1 - t^2), the
//    bias-gradient column (B's extra all-ones column), and per-column {sum, M2} partials of
//    the stored output for the next layer's BatchNorm, grouped per forward call (combined by
//    cgl_bn_apply, cgl_kernels.hip).
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
// In-launch rendezvous of the tiles_m workgroups of one column tile (fused BatchNorm).
// Published words are written with agent-scope atomic (sc1, write-through) stores and drained
// before the ticket; the ticket counter is monotonic (zero at workspace creation, every launch
// adds exactly n per column tile), so target = the next multiple of n above this workgroup's
// ticket and no per-call reset is needed; one lane polls relaxed with s_sleep, then ONE
// every reader loads the published words with agent-scope atomic (sc1) loads, so the poll needs
// no agent acquire (cdna_hip_programming.md Guideline 16, the all-sc1 form).  Requires the launch's workgroups co-resident (the
// planner checks the grid against the occupancy); the spin is bounded and a timeout sets *err.
__device__ __forceinline__ void cgl_rendezvous(unsigned int* cnt, unsigned int n, unsigned int* err) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // every wave's publish stores have landed
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned int old = __hip_atomic_fetch_add((cgl_gu32*)cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned int target = old - old % n + n;
    unsigned int spins = 0;
    while ((int)(__hip_atomic_load((cgl_gu32*)cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 21)) {
        __hip_atomic_store((cgl_gu32*)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    // every handed-off word is read with an sc1 (agent-scope atomic) load, so no agent acquire
    // (buffer_inv) is needed -- only the compiler must not hoist those loads above the poll
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  __syncthreads();
}
#define CGL_BN_MAXT 32     // row tiles per column tile a fused BatchNorm combines (tiles_m <= 32)
#define CGL_BN_STG 4       // staged partial items per thread: tiles_m x tile columns <= 1024
// dynamic LDS a fused-BatchNorm problem needs for its staged partials (bytes)
inline int cgl_bn_stage_bytes(int tiles_m, int ncw) { return tiles_m * ncw * 16; }

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
  static constexpr int S = CGL_GEMM_STAGES;
};

typedef __attribute__((address_space(3))) void cgl_lds_void;
#define CGL_GL_NS 2        // LDS ring depth of the staged main loop (measured: 2 beats 3 at 64 KB per workgroup)

template <int LAYOUT, int VEC, int TM, int TN, bool SK, bool GL, int DT = 0, bool BNF = false>
__device__ __forceinline__ void cgl_gemm_body(const CglGemmDesc* __restrict__ d, int bid, float* __restrict__ s_red,
                                              float* __restrict__ s_col, int* __restrict__ s_flag,
                                              float* __restrict__ s_bn, double* __restrict__ s_bnd) {
  constexpr int S = CglPipe<TM, TN>::S;
  const int M = d->M, N = d->N, K = d->K;
  const int WN = d->WN, WK = d->WK, WM = d->WM;
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
  const int KS = (SK && d->ksplit > 1) ? d->ksplit : 1;   // SK: the split-K instantiation
  const int local = bid - d->wg_begin;
  const int ntile = d->tiles_m * d->tiles_n;
  const int nwg = ntile * KS;
  int unit = local;
  if (nwg >= 16) {
    const int xcd = local & 7, pos = local >> 3, q = nwg >> 3, r = nwg & 7;
    unit = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
  }
  const int tile = unit / KS, kslice = unit - tile * KS;
  const int tn = tile / d->tiles_m, tm = tile % d->tiles_m;
  const int BM = 32 * TM * WM;
  const int m0 = tm * BM + wm * 32 * TM;            // first row of this wave's tile
  const int n0 = (tn * WN + wn) * 32 * TN;          // first column of this wave's tile

  // ---------------- main loop
  const int b_ones = (LAYOUT != 0) ? d->b_ones_col : 0;
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

  if constexpr (GL && LAYOUT != 2 && TM == 1 && TN == 1 && VEC && DT == CGL_DTYPE_F32) {
    // ---------------- LDS-staged main loop (glds): the waves of one K-slice share a ring of
    // CGL_GL_NS stages of 32 k, filled by global_load_lds_dwordx4 in whole 128-byte row segments
    // (8 rows per wave-instruction) instead of fragment-shaped loads that touch 32 rows per
    // instruction (those saturate the vector L1's tag lookups: TA_ADDR_STALLED_BY_TC, r02 PMC).
    //   A (k-contiguous): image [32 WM rows][32 k], row r's 16-byte piece p at p ^ ((r >> 1) & 7)
    //     (conflict-free ds_read_b128 of 8 consecutive k per lane half: the k-permuted fragment);
    //   B, NT (k-contiguous): the same image of 32 WN rows; NN (n-contiguous): k-major image
    //     [32 k][32 WN], fragments by ds_read_b32 (32 consecutive columns per lane half).
    // Rows / columns past M / N read clamped (valid) addresses and feed unstored outputs; k past
    // K (last stage only) reads clamped addresses and A's values there are zeroed.
    const int gw = WM * WN;
    const int na = 4 * WM, nb = 4 * WN, ninst = na + nb, per = ninst / gw;
    const int stg = ninst * 256;                          // floats per stage of one slice
    float* ring = s_red + wk * CGL_GL_NS * stg;
    const int nst = (K + 31) / 32;
    const int nsl = KS * WK, sl = kslice * WK + wk;
    const int sb = (sl * nst) / nsl, se = ((sl + 1) * nst) / nsl;
    const int cmax = (nst + nsl - 1) / nsl;
    const int arow0 = tm * BM, bcol0 = tn * WN * 32;     // first A row / B row (NT) or column (NN) of the tile
    const int ldb = d->b.ld;
    float* __restrict__ a_copy = d->a_copy;
    const bool do_copy = a_copy && tn == 0 && wn == 0 && (m0 + li) < M && (m0 + li) >= d->a_copy_row0;
    // this lane's global source of each of its fill instructions (instruction q = wmn + u gw)
    const float* src[8];
    int src_k[8];            // NT / A: offset of the piece in k; NN's B: k-row within the stage
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int q = min(wmn + u * gw, ninst - 1);
      if (q < na || LAYOUT == 0) {
        const bool isA = q < na;
        const int row = (isA ? q : q - na) * 8 + (lane >> 3);
        const int p = (lane & 7) ^ ((row >> 1) & 7);
        src[u] = isA ? cgl_row(d->a, min(arow0 + row, M - 1)) : cgl_row(d->b, min(bcol0 + row, N - 1));
        src_k[u] = 4 * p;
      } else {                                            // NN's B: k-major image
        const int e = (q - na) * 256 + 4 * (lane & 63);   // float index in the [32][32 WN] image
        const int kr = e / (32 * WN), col = e % (32 * WN);
        src[u] = d->b.p0 + min(bcol0 + col, nmem - 4);
        src_k[u] = kr;
      }
    }
    auto issue = [&](int s, int buf) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (u < per) {
          const int q = wmn + u * gw;
          const float* g;
          if (q < na || LAYOUT == 0)
            g = src[u] + min(s * 32 + src_k[u], K - 4);
          else
            g = src[u] + (long)min(s * 32 + src_k[u], K - 1) * ldb;
          __builtin_amdgcn_global_load_lds((const void*)g, (cgl_lds_void*)(ring + buf * stg + q * 256), 16, 0, 0);
        }
      }
    };
    const int arow = wm * 32 + li, asw = (arow >> 1) & 7;
    const int brow = wn * 32 + li, bsw = (brow >> 1) & 7;
    for (int j = 0; j < CGL_GL_NS - 1; ++j)
      if (sb + j < se) issue(sb + j, j);
    for (int it = 0; it < cmax; ++it) {
      const int s = sb + it;
      if (CGL_GL_NS > 2 && s + CGL_GL_NS - 2 < se) {
        // (CGL_GL_NS == 3: the next stage's `per` fills may stay in flight)
        switch (per) {
          case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
          case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
          case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
          default: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
        }
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      // (a full __syncthreads: it also orders the compiler's LDS reads after the barrier; with
      // CGL_GL_NS == 2 no fill is in flight here, so its vmcnt(0) costs nothing)
      __syncthreads();
      if (s + CGL_GL_NS - 1 < se) issue(s + CGL_GL_NS - 1, (it + CGL_GL_NS - 1) % CGL_GL_NS);
      if (s < se) {
        const float* la = ring + (it % CGL_GL_NS) * stg;
        const float* lb = la + na * 256;
        const int kleft = K - s * 32;                     // < 32 on a K-tail stage
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int p0 = 4 * c + 2 * lh;
          const f32x4 a0 = *(const f32x4*)(la + arow * 32 + 4 * (p0 ^ asw));
          const f32x4 a1 = *(const f32x4*)(la + arow * 32 + 4 * ((p0 + 1) ^ asw));
          float av[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
          float bv[8];
          if (LAYOUT == 0) {
            const f32x4 b0 = *(const f32x4*)(lb + brow * 32 + 4 * (p0 ^ bsw));
            const f32x4 b1 = *(const f32x4*)(lb + brow * 32 + 4 * ((p0 + 1) ^ bsw));
            bv[0] = b0[0]; bv[1] = b0[1]; bv[2] = b0[2]; bv[3] = b0[3];
            bv[4] = b1[0]; bv[5] = b1[1]; bv[6] = b1[2]; bv[7] = b1[3];
          } else {
#pragma unroll
            for (int q = 0; q < 8; ++q) bv[q] = lb[(16 * c + 8 * lh + q) * (32 * WN) + brow];
          }
          if (kleft < 32) {
#pragma unroll
            for (int q = 0; q < 8; ++q)
              if (16 * c + 8 * lh + q >= kleft) av[q] = 0.f;
          }
          if (do_copy) {
            float* dst = a_copy + (long)(m0 + li) * d->a_copy_ld + s * 32 + 16 * c + 8 * lh;
            if (kleft >= 16 * c + 8 * lh + 8) {
              *(gf4p)dst = f32x4{av[0], av[1], av[2], av[3]};
              *(gf4p)(dst + 4) = f32x4{av[4], av[5], av[6], av[7]};
            } else {
#pragma unroll
              for (int q = 0; q < 8; ++q)
                if (16 * c + 8 * lh + q < kleft) gst(dst + q, av[q]);
            }
          }
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            if (q % NX == 0)
              acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[q], bv[q], acc[0][0], 0, 0, 0);
            else
              accx[q % NX - 1] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[q], bv[q], accx[q % NX - 1], 0, 0, 0);
          }
        }
      }
    }
    __syncthreads();                        // the ring is reused by the split-K reduction below
  } else {
  const int nch = (K + CGL_GEMM_KCHUNK - 1) / CGL_GEMM_KCHUNK;
  // chunk range of this wave: slice kslice * WK + wk of KS * WK equal slices of the K chunks
  const int nsl = KS * WK, sl = kslice * WK + wk;
  const int cb = (sl * nch) / nsl, ce = ((sl + 1) * nch) / nsl;
  const int lda = d->a.ld, ldb = d->b.ld;
  float* __restrict__ a_copy = d->a_copy;

  // per-lane operand rows / columns of each block, clamped (always dereferenceable) bases
  const float* a_base[TM];
  const float* b_base[TN];
  bool b_is_ones[TN], do_copy[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int am = m0 + 32 * i + li;      // A row (kc) or A column (mn)
    a_base[i] = (LAYOUT != 2) ? cgl_row(d->a, min(am, M - 1)) : d->a.p0 + min(am, M - 1);
    do_copy[i] = (LAYOUT != 2) && a_copy && tn == 0 && wn == 0 && am < M && am >= d->a_copy_row0;
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int bc = n0 + 32 * j + li;      // B row (NT) or B column (NN/TN)
    b_is_ones[j] = b_ones && (bc == N - 1);
    b_base[j] = (LAYOUT == 0) ? cgl_row(d->b, min(bc, N - 1)) : d->b.p0 + max(0, min(bc, nmem - 1));
  }

  // Full chunks (k + 16 <= K) load without clamps and multiply without masks: rows / columns
  // past M / N come from clamped (valid) addresses and only feed accumulator rows / columns
  // that are never stored.  Only the K-tail chunk clamps its k and zeroes k >= K.
  auto load_chunk = [&](auto tail, int c, float (&A_)[TM][8], float (&B_)[TN][8]) {
    constexpr bool T = decltype(tail)::value;
    const int k = c * CGL_GEMM_KCHUNK + 8 * lh;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      if (LAYOUT == 2) {
        if (T) {
          cgl_ld_mn(a_base[i], lda, k, K, A_[i]);
        } else {
          gcfp q = (gcfp)a_base[i] + (long)k * lda;
#pragma unroll
          for (int j = 0; j < 8; ++j) A_[i][j] = q[(long)j * lda];
        }
      } else {
        if (T) {
          cgl_ld_kc<VEC>(a_base[i], k, K, A_[i]);
        } else if (VEC) {
          const f32x4 x = *(gcf4p)(a_base[i] + k), y = *(gcf4p)(a_base[i] + k + 4);
          A_[i][0] = x[0]; A_[i][1] = x[1]; A_[i][2] = x[2]; A_[i][3] = x[3];
          A_[i][4] = y[0]; A_[i][5] = y[1]; A_[i][6] = y[2]; A_[i][7] = y[3];
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) A_[i][j] = ((gcfp)a_base[i])[k + j];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if (LAYOUT == 0) {
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
  auto compute_chunk = [&](auto tail, int c, float (&A_)[TM][8], float (&B_)[TN][8]) {
    constexpr bool T = decltype(tail)::value;
    const int k = c * CGL_GEMM_KCHUNK + 8 * lh;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      if (T) cgl_mask(A_[i], true, k, K);
      if (do_copy[i]) {
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
  // loop body is branch-free (refills past the end re-load the last full chunk, harmlessly), so
  // every s_waitcnt waits for exactly the set it consumes.
  const int cfull = min(ce, K / CGL_GEMM_KCHUNK);   // end of this wave's full chunks
  std::integral_constant<bool, false> full;
  std::integral_constant<bool, true> tailc;
  if (cb < cfull) {
    float xa[S][TM][8], xb[S][TN][8];
#pragma unroll
    for (int s = 0; s < S; ++s) load_chunk(full, min(cb + s, cfull - 1), xa[s], xb[s]);
    int c = cb;
    for (; c + S <= cfull; c += S) {
#pragma unroll
      for (int s = 0; s < S; ++s) {
        compute_chunk(full, c + s, xa[s], xb[s]);
        load_chunk(full, min(c + s + S, cfull - 1), xa[s], xb[s]);
      }
    }
#pragma unroll
    for (int s = 0; s < S - 1; ++s)
      if (c + s < cfull) compute_chunk(full, c + s, xa[s], xb[s]);
  }
  if (cfull < ce) {   // the K tail (at most one chunk, owned by the last k-group)
    float xa[TM][8], xb[TN][8];
    load_chunk(tailc, cfull, xa, xb);
    compute_chunk(tailc, cfull, xa, xb);
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
      const float bb = d->bias ? gld(d->bias + col) : 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        float* v = (float*)&acc[i][j];
        if (d->bias) {
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] += bb;
        }
        if (d->act == CGL_EPI_ACT_LEAKY) {
          const float sl = d->slope;
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * sl;
        } else if (d->act == CGL_EPI_ACT_TANH) {
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = tanhf(v[r]);   // (double tanh here costs ~4 us on G L4)
        } else if (d->act == CGL_EPI_ACT_SIGMOID) {
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = 1.f / (1.f + expf(-v[r]));
        }
        if (d->mask_ref) {
          const float sl = d->slope;
          float ref[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = min(rbase + 32 * i + (r & 3) + 8 * (r >> 2), M - 1);
            ref[r] = gld(d->mask_ref + (long)row * d->mask_ld + col);
          }
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = ref[r] > 0.f ? v[r] : v[r] * sl;
        }
        if (d->tanh_ref) {
          float t[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = min(rbase + 32 * i + (r & 3) + 8 * (r >> 2), M - 1);
            t[r] = gld(d->tanh_ref + (long)row * d->tanh_ld + col);
          }
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] = cgl_dtanh(v[r], t[r]);
        }
      }
    }
  }

  // ---------------- fused BatchNorm1d backward (bn_fuse 2): C = dZ of the BatchNorm below
  // (torch's batch_norm_backward, train mode, as cgl_bn_bwd):
  //   dy = leaky'(post) * acc,  S = sum dy,  D = sum (y - mean) dy   (per column, over all M rows)
  //   dZ = (dy - S / M - (y - mean) D invstd^2 / M) invstd gamma,  dgamma = D invstd,  dbeta = S
  if (BNF && d->bn_fuse == 2) {   // (BNF: only the fused-BatchNorm instantiation carries these paths)
    const float sl = d->slope;
    float dy[TM][TN][16], yc[TM][TN][16];
    const int ldp = d->bn_ld_post;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int colc = min(n0 + 32 * j + li, N - 1);
      const float mu = gld(d->bn_mean + colc);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        float po[16], yv[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = min(rbase + 32 * i + (r & 3) + 8 * (r >> 2), M - 1);
          po[r] = gld(d->bn_post + (long)row * ldp + colc);
          yv[r] = gld(d->bn_y + (long)row * ldp + colc);
        }
        const float* v = (const float*)&acc[i][j];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          dy[i][j][r] = po[r] > 0.f ? v[r] : v[r] * sl;
          yc[i][j][r] = yv[r] - mu;
        }
      }
    }
    // tile partials per column: lane rows (16 per block) -> lane halves -> waves of the column
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const bool colok = n0 + 32 * j + li < N;
      double S = 0.0, D = 0.0;
      if (owner && colok) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = rbase + 32 * i + (r & 3) + 8 * (r >> 2);
            if (row < M) {
              S += (double)dy[i][j][r];
              D += (double)(yc[i][j][r] * dy[i][j][r]);
            }
          }
      }
      S += __shfl_xor(S, 32);
      D += __shfl_xor(D, 32);
      if (owner && lh == 0) {
        s_bnd[(((wm * WN + wn) * TN + j) * 32 + li) * 2] = S;
        s_bnd[(((wm * WN + wn) * TN + j) * 32 + li) * 2 + 1] = D;
      }
    }
    __syncthreads();
    if (owner && wm == 0 && lh == 0) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n0 + 32 * j + li;
        double S = 0.0, D = 0.0;
        for (int q = 0; q < WM; ++q) {
          S += s_bnd[(((q * WN + wn) * TN + j) * 32 + li) * 2];
          D += s_bnd[(((q * WN + wn) * TN + j) * 32 + li) * 2 + 1];
        }
        if (col < N) {
          cgl_pubd(d->bn_dpart + ((long)tm * N + col) * 2, S);
          cgl_pubd(d->bn_dpart + ((long)tm * N + col) * 2 + 1, D);
        }
      }
    }
    cgl_rendezvous(d->rv_count + tn, (unsigned int)d->tiles_m, d->err);
    // every column of the workgroup tile: the tiles_m partials staged through LDS (one round trip,
    // few registers), then summed in tile order
    const int ncw = WN * TN * 32, c0 = tn * WN * TN * 32;
    float* s_gm = s_bn;          // [ncw]: S / M
    float* s_k = s_bn + 128;     // [ncw]: D invstd^2 / M
    {
      const int nt = d->tiles_m, items = nt * ncw;
      unsigned long long* stg = (unsigned long long*)s_red;    // [nt][ncw][2]
      unsigned long long v0[CGL_BN_STG], v1[CGL_BN_STG];
#pragma unroll
      for (int u = 0; u < CGL_BN_STG; ++u) {
        const int q = min(tid + 256 * u, items - 1);
        const int t = q / ncw, col = min(c0 + q % ncw, N - 1);
        v0[u] = cgl_ld64(d->bn_dpart + ((long)t * N + col) * 2);
        v1[u] = cgl_ld64(d->bn_dpart + ((long)t * N + col) * 2 + 1);
      }
#pragma unroll
      for (int u = 0; u < CGL_BN_STG; ++u) {
        const int q = tid + 256 * u;
        if (q < items) {
          stg[2 * q] = v0[u];
          stg[2 * q + 1] = v1[u];
        }
      }
    }
    __syncthreads();
    if (tid < ncw) {
      const int col = min(c0 + tid, N - 1);
      const int nt = d->tiles_m;
      const unsigned long long* stg = (const unsigned long long*)s_red;
      double S = 0.0, D = 0.0;
      for (int t = 0; t < nt; ++t) {
        S += __longlong_as_double((long long)stg[2 * (t * ncw + tid)]);
        D += __longlong_as_double((long long)stg[2 * (t * ncw + tid) + 1]);
      }
      const float invstd = gld(d->bn_invstd + col);
      s_k[tid] = (float)D * invstd * invstd / M;
      s_gm[tid] = (float)(S / M);
      if (tm == 0 && c0 + tid < N) {
        gst(d->bn_g_gamma + col, (float)(D * (double)invstd));
        gst(d->bn_g_beta + col, (float)S);
      }
    }
    __syncthreads();
    if (owner) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n0 + 32 * j + li;
        if (col >= N) continue;
        const int cl = col - c0;
        const float invstd = gld(d->bn_invstd + col), w = gld(d->bn_gamma + col);
        const float gm = s_gm[cl], k = s_k[cl];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = rbase + 32 * i + (r & 3) + 8 * (r >> 2);
            if (row < M) gst(d->C + (long)row * d->ldc + col, (dy[i][j][r] - gm - yc[i][j][r] * k) * invstd * w);
          }
      }
    }
    return;
  }

  // forward BatchNorm partials of the stored output: per column, per group slot {sum, M2}
  // over the workgroup's BM rows (two-pass: tile-slot sum, then M2 about the tile-slot mean)
  if (d->stat_part) {
    const int gr = d->stat_gr;
    const int trow0 = tm * BM;
    const int gfirst = trow0 / gr;
    const int gsplit = (gfirst + 1) * gr;   // first row of slot 1 (a tile spans <= 2 groups)
    float part[TN][2][2];
    for (int s = 0; s < 2; ++s) {
      const int ra = max(trow0, (gfirst + s) * gr), rb = min(min(trow0 + BM, M), (gfirst + s + 1) * gr);
      const int cnt = rb - ra;
      float tot[TN], mean[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const bool colok = n0 + 32 * j + li < N;
        float sum = 0.f;
        if (owner && colok) {
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            const float* v = (const float*)&acc[i][j];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int row = rbase + 32 * i + (r & 3) + 8 * (r >> 2);
              if (row < M && (row >= gsplit) == (s == 1)) sum += v[r];
            }
          }
        }
        sum += __shfl_xor(sum, 32);
        if (owner && lh == 0) s_col[((wm * WN + wn) * TN + j) * 32 + li] = sum;
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        float t = 0.f;
        for (int q = 0; q < WM; ++q) t += s_col[((q * WN + wn) * TN + j) * 32 + li];
        tot[j] = t;
        mean[j] = cnt > 0 ? t / cnt : 0.f;
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const bool colok = n0 + 32 * j + li < N;
        float q2 = 0.f;
        if (owner && colok) {
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            const float* v = (const float*)&acc[i][j];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int row = rbase + 32 * i + (r & 3) + 8 * (r >> 2);
              if (row < M && (row >= gsplit) == (s == 1)) {
                const float dd = v[r] - mean[j];
                q2 += dd * dd;
              }
            }
          }
        }
        q2 += __shfl_xor(q2, 32);
        if (owner && lh == 0) s_col[((wm * WN + wn) * TN + j) * 32 + li] = q2;
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        float qt = 0.f;
        for (int q = 0; q < WM; ++q) qt += s_col[((q * WN + wn) * TN + j) * 32 + li];
        part[j][s][0] = cnt > 0 ? tot[j] : 0.f;
        part[j][s][1] = cnt > 0 ? qt : 0.f;
      }
      __syncthreads();
    }
    if (owner && wm == 0 && lh == 0) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n0 + 32 * j + li;
        if (col < N) {
          for (int s = 0; s < 2; ++s) {
            float* p = d->stat_part + ((long)(tm * 2 + s) * N + col) * 2;
            if (d->bn_fuse == 1) {
              cgl_pub2f(p, part[j][s][0], part[j][s][1]);
            } else {
              gst(p, part[j][s][0]);
              gst(p + 1, part[j][s][1]);
            }
          }
        }
      }
    }
  }

  // ---------------- fused BatchNorm1d forward (bn_fuse 1): C = Y (the Linear output, kept for
  // the backward), act = LeakyReLU(BN(Y)) with the statistics of the Y rows' forward call (group
  // of stat_gr rows), combined from every row tile's published {sum, M2} partials exactly as
  // cgl_bn_apply does (tile order, double, Chan); row tile 0 writes save_mean / save_invstd and
  // updates the running statistics group by group (the reference's forward-call order)
  if (BNF && d->bn_fuse == 1) {
    cgl_rendezvous(d->rv_count + tn, (unsigned int)d->tiles_m, d->err);
    const int gr = d->stat_gr;
    const int ng = (M + gr - 1) / gr;          // <= 2 (planner)
    const int ncw = WN * TN * 32, c0 = tn * WN * TN * 32;
    float* s_sc = s_bn;            // [2][128]
    float* s_sh = s_bn + 256;      // [2][128]
    double* s_mu = s_bnd;          // [2][128]
    double* s_m2 = s_bnd + 256;    // [2][128]
    {
      // stage every row tile's {sum, M2} pair of both group slots for the tile's columns (one round
      // trip): stg[slot][t][c]
      const int nt = d->tiles_m, items = 2 * nt * ncw;
      unsigned long long* stg = (unsigned long long*)s_red;
      unsigned long long v[2 * CGL_BN_STG];
#pragma unroll
      for (int u = 0; u < 2 * CGL_BN_STG; ++u) {
        const int q = min(tid + 256 * u, items - 1);
        const int sl2 = q / (nt * ncw), t = (q / ncw) % nt, col = min(c0 + q % ncw, N - 1);
        v[u] = cgl_ld64(d->stat_part + ((long)(t * 2 + sl2) * N + col) * 2);
      }
#pragma unroll
      for (int u = 0; u < 2 * CGL_BN_STG; ++u) {
        const int q = tid + 256 * u;
        if (q < items) stg[q] = v[u];
      }
    }
    __syncthreads();
    int n_g = 0;
    if (tid < ncw * ng) {
      const int cl = tid % ncw, g = tid / ncw;
      const int col = min(c0 + cl, N - 1);
      const int r0 = g * gr, r1 = min(r0 + gr, M);
      n_g = r1 - r0;
      const int t0 = r0 / BM, t1 = (r1 - 1) / BM;
      const int nt = t1 - t0 + 1;
      const unsigned long long* stg = (const unsigned long long*)s_red;
      auto pr = [&](int j) {
        const int t = t0 + j;
        const int slot = (t * BM < r0) ? 1 : 0;   // tile starts in the previous group
        return stg[(slot * d->tiles_m + t) * ncw + cl];
      };
      double sm = 0.0;
      for (int j = 0; j < nt; ++j) sm += (double)__uint_as_float((unsigned int)pr(j));
      const double mu = sm / n_g;
      double m2 = 0.0;
      for (int j = 0; j < nt; ++j) {
        const int t = t0 + j;
        const int c = min((t + 1) * BM, r1) - max(t * BM, r0);
        const unsigned long long p = pr(j);
        const double dd = (double)__uint_as_float((unsigned int)p) / c - mu;
        m2 += (double)__uint_as_float((unsigned int)(p >> 32)) + c * dd * dd;
      }
      const double invstd = 1.0 / sqrt(m2 / n_g + d->bn_eps);
      const float sc = (float)invstd * gld(d->bn_gamma + col);
      s_sc[g * 128 + cl] = sc;
      s_sh[g * 128 + cl] = gld(d->bn_beta + col) - (float)mu * sc;
      s_mu[g * 128 + cl] = mu;
      s_m2[g * 128 + cl] = m2;
      if (tm == 0 && c0 + cl < N && d->bn_save_mean) {
        gst(d->bn_save_mean + (long)g * N + col, (float)mu);
        gst(d->bn_save_invstd + (long)g * N + col, (float)invstd);
      }
    }
    __syncthreads();
    if (tm == 0 && tid < ncw && c0 + tid < N && d->bn_run_mean) {
      const int col = c0 + tid;
      const double mom = d->bn_momentum;
      float rm = gld(d->bn_run_mean + col), rv = gld(d->bn_run_var + col);
      for (int g = 0; g < ng; ++g) {
        const int n = min((g + 1) * gr, M) - g * gr;
        rm = (float)(mom * s_mu[g * 128 + tid] + (1.0 - mom) * (double)rm);
        rv = (float)(mom * (s_m2[g * 128 + tid] / (n - 1)) + (1.0 - mom) * (double)rv);
      }
      gst(d->bn_run_mean + col, rm);
      gst(d->bn_run_var + col, rv);
    }
    if (owner) {
      const float sl = d->slope;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n0 + 32 * j + li;
        if (col >= N) continue;
        const int cl = col - c0;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const float* v = (const float*)&acc[i][j];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = rbase + 32 * i + (r & 3) + 8 * (r >> 2);
            if (row < M) {
              const int g = row >= gr ? 1 : 0;
              const float x = fmaf(v[r], s_sc[g * 128 + cl], s_sh[g * 128 + cl]);
              gst(d->C + (long)row * d->ldc + col, v[r]);
              gst(d->bn_act + (long)row * d->bn_ld_act + col, x > 0.f ? x : x * sl);
            }
          }
        }
      }
    }
    return;
  }

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
          if (d->bias_out) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int row = rbase + 32 * i + (r & 3) + 8 * (r >> 2);
              if (row < M) gst(d->bias_out + row, v[r]);
            }
          }
        } else {
          float* __restrict__ C = d->C;
          const int ldc = d->ldc;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = rbase + 32 * i + (r & 3) + 8 * (r >> 2);
            if (row < M) gst(C + (long)row * ldc + col, v[r]);
          }
        }
      }
    }
  }
}

// One kernel per per-wave block shape (TM x TN), shared by every GEMM of the step; a grouped
// launch may mix layouts (e.g. the weight gradient (TN) and the input gradient (NN) of one
// layer side by side).  Separate symbols keep the 1x1 variant's register budget (and so its
// occupancy) independent of the 2x2 variant's.
// Dynamic LDS: split-K partials of the waves with wk > 0.
// BNF: the instantiation that carries the (opt-in) fused-BatchNorm epilogues (bn_fuse 1 / 2); the
// default instantiations compile them out, so their register budget is the plain GEMM's.
template <int TM, int TN, bool SK = false, bool GL = false, int DT = CGL_DTYPE_F32, bool BNF = false>
__global__ __launch_bounds__(CGL_GEMM_THREADS) void cgl_gemm_f32(const CglGemmDesc* __restrict__ descs, int ndesc) {
  extern __shared__ float cgl_dyn_lds[];
  __shared__ float s_col[4 * TN * 32];          // per-column reductions across waves (WM WN <= 4)
  __shared__ int s_flag[1];                     // split-K: this workgroup reduces its tile
  __shared__ float s_bn[512];                   // fused BatchNorm: per-column tables
  __shared__ double s_bnd[4 * TN * 32 * 2 > 512 ? 4 * TN * 32 * 2 : 512];
  float* s_red = cgl_dyn_lds;
  const int bid = blockIdx.x;
  int di = 0;
  for (int q = 1; q < ndesc; ++q)
    if (bid >= descs[q].wg_begin) di = q;
  const CglGemmDesc* __restrict__ d = descs + di;
  const int layout = d->layout;
  // VEC: every operand allows 16-byte loads along its contiguous dimension
  const int vec = d->a_vec && d->b_vec;
#define CGL_BODY(L)                                               \
  do {                                                            \
    if (vec)                                                      \
      cgl_gemm_body<L, 1, TM, TN, SK, GL, DT, BNF>(d, bid, s_red, s_col, s_flag, s_bn, s_bnd);    \
    else                                                          \
      cgl_gemm_body<L, 0, TM, TN, SK, GL, DT, BNF>(d, bid, s_red, s_col, s_flag, s_bn, s_bnd);    \
  } while (0)
  if (layout == 0)
    CGL_BODY(0);
  else if (layout == 1)
    CGL_BODY(1);
  else
    CGL_BODY(2);
#undef CGL_BODY
}

// Host helper: dynamic LDS bytes of one problem's split-K partials.
// LDS ring of the staged main loop (GL launches, 1x1 blocks, layouts 0 / 1 with 16-byte operands)
inline bool cgl_gemm_gl_ok(const CglGemmDesc& d) {
  return d.layout != 2 && d.TM == 1 && d.TN == 1 && d.a_vec && d.b_vec && d.ksplit <= 1 && !d.b_ones_col &&
         d.WM * d.WN * d.WK == 4;
}
inline int cgl_gemm_gl_bytes(const CglGemmDesc& d) {
  return cgl_gemm_gl_ok(d) ? d.WK * CGL_GL_NS * (4 * d.WM + 4 * d.WN) * 1024 : 0;
}
inline int cgl_gemm_stage_bytes(const CglGemmDesc& d, bool gl = false) {
  const int sk0 = (d.WK > 1) ? d.WM * d.WN * (d.WK - 1) * d.TM * d.TN * 16 * 64 * 4 : 0;
  const int glb = gl ? cgl_gemm_gl_bytes(d) : 0;
  const int sk = sk0 > glb ? sk0 : glb;
  const int bn = d.bn_fuse ? cgl_bn_stage_bytes(d.tiles_m, d.WN * d.TN * 32) : 0;
  return sk > bn ? sk : bn;
}

// Host helpers: workgroups of one problem, and the split-K partial floats it needs.
inline int cgl_gemm_wgs(const CglGemmDesc& d) { return d.tiles_m * d.tiles_n * (d.ksplit > 1 ? d.ksplit : 1); }
inline long cgl_gemm_kpart_floats(const CglGemmDesc& d) {
  return d.ksplit > 1 ? (long)d.ksplit * d.tiles_m * d.tiles_n * d.WM * d.WN * d.TM * d.TN * 16 * 64 : 0;
}
