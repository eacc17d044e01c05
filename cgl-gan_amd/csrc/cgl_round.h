// Device code of the round prologue (per-round scalars, z draw, real-batch sampler, operand packing) and
// its fusion with G's first GEMM (cgl_gemm_pro).  Included by cgl_runtime.hip (which launches them) and by
// the GEMM-instantiation translation units (cgl_gemm_inst.hip, which compile cgl_gemm_pro's instances).
#pragma once
#include "cgl_internal.h"

namespace {
// Round prologue: block 0 writes the round's scalars, the next nb_norm blocks draw z, the
// last blocks draw the real-row indices of this round's local D steps.  Every block reads the
// completed-round counter, which only the G-Adam tail (a later launch) advances.
// The round prologue's last blocks pack operands into the GEMMs' fragment layout (CglOpPackJob): thread
// t of a job writes packed float4 t, i.e. (row block, chunk, half, lane) of P(X; R, K); a transposed
// source is read along its contiguous rows (the lanes of a block span 32 consecutive r).
__device__ __forceinline__ void cgl_pack_job(const CglOpPackJob& J, long t) {
  const int Kc = (J.K + 15) >> 4;
  const long n4 = (long)((J.R + 31) >> 5) * Kc * 128;
  if (t >= n4) return;
  const int l = (int)(t & 63), h = (int)((t >> 6) & 1);
  const long q = t >> 7;
  const int c = (int)(q % Kc), rb = (int)(q / Kc);
  const int r = rb * 32 + (l & 31), k0 = c * 16 + 8 * (l >> 5) + 4 * h;
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  if (r < J.R) {
    if (J.trans) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (k0 + e < J.K) v[e] = gld(J.src + (long)(k0 + e) * J.ld + r);
    } else if (k0 + 3 < J.K && ((J.ld | J.K) & 3) == 0) {
      v = *(gcf4p)(J.src + (long)r * J.ld + k0);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (k0 + e < J.K) v[e] = gld(J.src + (long)r * J.ld + k0 + e);
    }
  }
  *(gf4p)(J.dst + t * 4) = v;
}

__device__ __forceinline__ void cgl_round_prologue_at(int bid, int nblk, const CglBeginArgs& a, float* z, long nz,
                                                      unsigned long long zseed, int nb_norm, int* idx, int epoch,
                                                      int br, int n, unsigned long long sseed, const CglOpPack& pk) {
  const int done = a.st->round;
  const int pk0 = nblk - pk.blocks;     // the packing blocks come last
  if (bid >= pk0) {
    const int b = bid - pk0;
    int j = 0;
    for (int q = 1; q < pk.nj; ++q)
      if (b >= pk.j[q].blk_begin) j = q;
    cgl_pack_job(pk.j[j], (long)(b - pk.j[j].blk_begin) * 256 + threadIdx.x);
    return;
  }
  if (bid == 0) {
    if (threadIdx.x == 0) cgl_begin_at(a, done + 1);
    return;
  }
  if (bid <= nb_norm) {
    cgl_normal_at((long)(bid - 1) * 256 + threadIdx.x, z, nz, zseed, (uint32_t)(done + 1), 0);
    return;
  }
  // DataLoader(shuffle=True) over the n resident rows (capgan.py:282, 326-331): each pass is a fresh
  // keyed permutation cut into ceil(n / br) batches, the last one short (n mod br rows); local D step
  // e of round `done` takes batch done * epoch + e.  Rows past a short batch index a valid dummy row
  // (no loss, no gradient: the head's n0_dev)
  const int t = (bid - 1 - nb_norm) * 256 + threadIdx.x;
  if (t >= epoch * br) return;
  const int e = t / br, row = t - e * br;
  const long nb = (n + br - 1) / br;
  const long bpos = (long)done * epoch + e;
  const uint32_t pass = (uint32_t)(bpos / nb);
  const long b = bpos % nb;
  const long j = b * br + row;
  idx[t] = (int)cgl_permute((uint32_t)(j < n ? j : n - 1), (uint32_t)n,
                            (uint32_t)sseed ^ (pass * 0x85ebca6bu + 0x1234567u));
  if (row == 0) a.st->real_rows[e] = (int)(n - b * br < br ? n - b * br : br);
}

#ifndef CGL_GEMM_PART_TU
// The packing jobs alone (cgl_gan_sync_params): after G's parameters were written from outside the round
// (load, initialisation, a Cloud FedAvg) while the packed copies are maintained by the G Adam launch.
__global__ __launch_bounds__(256) void cgl_pack_all(CglOpPack pk) {
  const int b = blockIdx.x;
  int j = 0;
  for (int q = 1; q < pk.nj; ++q)
    if (b >= pk.j[q].blk_begin) j = q;
  cgl_pack_job(pk.j[j], (long)(b - pk.j[j].blk_begin) * 256 + threadIdx.x);
}

// cgl_bn_apply with operand-packing jobs riding in blocks [nbn, grid) (plan_pack_carriers); blocks [0, nbn) are the
// BatchNorm apply's (gx, nbn / gx) grid, row-major
__global__ __launch_bounds__(256) void cgl_bn_apply_pk(const CglBnApplyDesc d, int gx, int nbn, const CglOpPack pk) {
  const int b = blockIdx.x;
  if (b < nbn) {
    cgl_bn_apply_body(&d, b % gx, b / gx);
    return;
  }
  const int q = b - nbn;
  int j = 0;
  for (int i = 1; i < pk.nj; ++i)
    if (q >= pk.j[i].blk_begin) j = i;
  cgl_pack_job(pk.j[j], (long)(q - pk.j[j].blk_begin) * 256 + threadIdx.x);
}

// a deferred cgl_head_loss (its partials reduced by the next launch) with packing jobs in blocks [nhead, grid)
__global__ __launch_bounds__(256) void cgl_head_loss_pk(const CglHeadDesc d, int nhead, const CglOpPack pk) {
  const int b = blockIdx.x;
  if (b < nhead) {
    cgl_head_loss_body(&d, b, nhead);
    return;
  }
  const int q = b - nhead;
  int j = 0;
  for (int i = 1; i < pk.nj; ++i)
    if (q >= pk.j[i].blk_begin) j = i;
  cgl_pack_job(pk.j[j], (long)(q - pk.j[j].blk_begin) * 256 + threadIdx.x);
}

// G's Adam with the operand packing of the next round (CglAdamPack, plan flag pack_adam): the weight matrices
// that carry packing jobs are updated in 4 x 4 tiles -- one thread loads 4 rows x 4 columns of p / g / m / v
// with 16-byte loads, applies cgl_adam_update to each of the 16 values (the arithmetic of cgl_adam_at, element
// by element), stores them back and writes the updated values straight into the packed forward operand
// P(W; R, K) (4 consecutive k of a row = one float4) and the packed transposed operand P(W^T; K, R) (4
// consecutive r of a column = one float4, transposed in registers).  Every other parameter (biases, BatchNorm,
// unpacked layers, alignment padding) goes through cgl_adam_at over the element ranges.  The round prologue
// then no longer re-packs G every round (25 MB of traffic per round, profiles/r04_traffic.json).
#define CGL_APK_MAXT 8
#define CGL_APK_MAXR 10
struct CglAdamPackTile {
  long off;               // first float of W [R][K] in the flat buffer
  int R, K;               // R % 4 == K % 4 == 0
  float* fwd;             // P(W; R, K), or null
  float* trn;             // P(W^T; K, R), or null
  int blk_begin;
  int t32;                // 1: 32 x 64 workgroup tiles through LDS (K % 8 == 0), 0: 4 x 4 thread tiles
};
struct CglAdamPack {
  int nt, nr, tile_blocks;
  CglAdamPackTile t[CGL_APK_MAXT];
  long r0[CGL_APK_MAXR], r1[CGL_APK_MAXR];   // element ranges [r0, r1) of the flat buffer
  int rblk[CGL_APK_MAXR];                     // first block of each range (after the tile blocks)
};

__device__ __forceinline__ void cgl_adam_tile_at(const CglAdamArgs& a, const CglAdamPackTile& T, long t) {
  const int kq = T.K >> 2;
  if (t >= (long)(T.R >> 2) * kq) return;
  const int r = (int)(t / kq) * 4, k = (int)(t % kq) * 4;
  const long e0 = T.off + (long)r * T.K + k;
  const float ss = a.step_size ? gld(a.step_size) : a.step_size_v;
  const float bc = a.bc2sqrt ? gld(a.bc2sqrt) : a.bc2sqrt_v;
  f32x4 P[4], G[4], M[4], V[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const long e = e0 + (long)i * T.K;
    P[i] = *(gcf4p)(a.p + e);
    G[i] = *(gcf4p)(a.g + e);
    M[i] = *(gcf4p)(a.m + e);
    V[i] = *(gcf4p)(a.v + e);
  }
  bool upd = true;
  if (a.scale) {
    const float inv = (float)(1.0 / (double)gld(a.scale));
    upd = *(const CGL_GLOBAL unsigned int*)a.found == 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) G[i][j] = G[i][j] * inv;
      *(gf4p)(a.g + e0 + (long)i * T.K) = G[i];
    }
  }
  if (upd) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float pp = P[i][j], mm = M[i][j], vv = V[i][j];
        cgl_adam_update(pp, G[i][j], mm, vv, ss, bc, a.b2, a.w1, a.w2, a.eps);
        P[i][j] = pp;
        M[i][j] = mm;
        V[i][j] = vv;
      }
      const long e = e0 + (long)i * T.K;
      *(gf4p)(a.m + e) = M[i];
      *(gf4p)(a.v + e) = V[i];
      *(gf4p)(a.p + e) = P[i];
    }
  }
  if (T.fwd) {
    const int kc = (T.K + 15) >> 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) *(gf4p)(T.fwd + cgl_pk_off(r + i, k, kc)) = P[i];
  }
  if (T.trn) {
    const int kc = (T.R + 15) >> 4;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      *(gf4p)(T.trn + cgl_pk_off(k + j, r, kc)) = f32x4{P[0][j], P[1][j], P[2][j], P[3][j]};
  }
}

// The same update for a 32-row x 64-column tile of W per workgroup (t32): thread (ri = tid / 8, 8 consecutive
// columns) loads its row segment with 16-byte loads (a row's 64 columns = 256 contiguous bytes), updates, stores
// p / m / v back, and drops the new values into LDS at their packed positions; the tile's forward image P(W) is
// then 4 consecutive 2 KB blocks (chunks k0 / 16 ..) and its transposed image P(W^T) 2 x 2 blocks, each written
// with contiguous 16-byte stores.  Positions past R / K inside a block hold zeros (the packing's padding).
__device__ __forceinline__ void cgl_adam_tile32_at(const CglAdamArgs& a, const CglAdamPackTile& T, int t,
                                                   float* s_f, float* s_t) {
  const int nkt = (T.K + 63) >> 6;
  const int rb = t / nkt, k0 = (t - rb * nkt) * 64;
  const int tid = threadIdx.x, ri = tid >> 3, kq = (tid & 7) * 8;
  const int r = rb * 32 + ri, k = k0 + kq;
  const bool ok = r < T.R && k < T.K;            // (K % 8 == 0: the 8 columns are all in or all out)
  const long e0 = T.off + (long)min(r, T.R - 1) * T.K + min(k, T.K - 8);
  const float ss = a.step_size ? gld(a.step_size) : a.step_size_v;
  const float bc = a.bc2sqrt ? gld(a.bc2sqrt) : a.bc2sqrt_v;
  f32x4 P[2], G[2], M[2], V[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    P[h] = *(gcf4p)(a.p + e0 + 4 * h);
    G[h] = *(gcf4p)(a.g + e0 + 4 * h);
    M[h] = *(gcf4p)(a.m + e0 + 4 * h);
    V[h] = *(gcf4p)(a.v + e0 + 4 * h);
  }
  bool upd = true;
  if (a.scale) {
    const float inv = (float)(1.0 / (double)gld(a.scale));
    upd = *(const CGL_GLOBAL unsigned int*)a.found == 0u;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int j = 0; j < 4; ++j) G[h][j] = G[h][j] * inv;
      if (ok) *(gf4p)(a.g + e0 + 4 * h) = G[h];
    }
  }
  if (upd) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float pp = P[h][j], mm = M[h][j], vv = V[h][j];
        cgl_adam_update(pp, G[h][j], mm, vv, ss, bc, a.b2, a.w1, a.w2, a.eps);
        P[h][j] = pp;
        M[h][j] = mm;
        V[h][j] = vv;
      }
      if (ok) {
        *(gf4p)(a.m + e0 + 4 * h) = M[h];
        *(gf4p)(a.v + e0 + 4 * h) = V[h];
        *(gf4p)(a.p + e0 + 4 * h) = P[h];
      }
    }
  }
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const f32x4 v = ok ? P[h] : z;
    const int kk = kq + 4 * h;
    // forward image: ((kk / 16) * 2 + (kk / 4) % 2) * 256 + (ri + 32 ((kk / 8) % 2)) * 4 + kk % 4
    *(f32x4*)(s_f + ((kk >> 4) * 2 + ((kk >> 2) & 1)) * 256 + (ri + 32 * ((kk >> 3) & 1)) * 4) = v;
    // transposed image: region kk / 32, then ((ri / 16) * 2 + (ri / 4) % 2) * 256 + (kk % 32 + 32 ((ri / 8) % 2)) * 4
    // + ri % 4
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = kk + j;
      s_t[(c >> 5) * 1024 + ((ri >> 4) * 2 + ((ri >> 2) & 1)) * 256 + ((c & 31) + 32 * ((ri >> 3) & 1)) * 4 + (ri & 3)] =
          v[j];
    }
  }
  __syncthreads();
  const int q = tid * 8;     // this thread's 8 floats of each 2048-float image
  if (T.fwd) {
    const int kc = (T.K + 15) >> 4;
    if ((k0 >> 4) + (q >> 9) < kc) {
      float* dst = T.fwd + ((long)rb * kc + (k0 >> 4)) * 512 + q;
      *(gf4p)dst = *(const f32x4*)(s_f + q);
      *(gf4p)(dst + 4) = *(const f32x4*)(s_f + q + 4);
    }
  }
  if (T.trn) {
    const int kc = (T.R + 15) >> 4, rbt = (k0 >> 5) + (q >> 10), ct = 2 * rb + ((q >> 9) & 1);
    if (rbt < ((T.K + 31) >> 5) && ct < kc) {
      float* dst = T.trn + ((long)rbt * kc + ct) * 512 + (q & 511);
      *(gf4p)dst = *(const f32x4*)(s_t + q);
      *(gf4p)(dst + 4) = *(const f32x4*)(s_t + q + 4);
    }
  }
}

__global__ __launch_bounds__(256) void cgl_adam_pack(CglAdamArgs a, CglAdamPack pk, CglStepState* st, int tail) {
  __shared__ float s_img[2][2048];
  if (cgl_adam_zblock(a, st)) return;
  const int b = blockIdx.x;
  if (b < pk.tile_blocks) {
    int j = 0;
    for (int q = 1; q < pk.nt; ++q)
      if (b >= pk.t[q].blk_begin) j = q;
    if (pk.t[j].t32)
      cgl_adam_tile32_at(a, pk.t[j], b - pk.t[j].blk_begin, s_img[0], s_img[1]);
    else
      cgl_adam_tile_at(a, pk.t[j], (long)(b - pk.t[j].blk_begin) * 256 + threadIdx.x);
  } else {
    int j = 0;
    for (int q = 1; q < pk.nr; ++q)
      if (b >= pk.rblk[q]) j = q;
    const long i = pk.r0[j] + (long)(b - pk.rblk[j]) * 256 + threadIdx.x;
    if (i < pk.r1[j]) {
      CglAdamArgs e = a;
      e.n = pk.r1[j];
      cgl_adam_at(e, st, 0, i);
    }
  }
  if (tail && b == 0 && threadIdx.x == 0) {   // the round's scalar tail, as cgl_adam_at's thread 0
    cgl_round_tail(st);
    if (a.scale) st->scaler_pending = 1;
  }
}

__global__ __launch_bounds__(256) void cgl_round_prologue(CglBeginArgs a, float* z, long nz, unsigned long long zseed,
                                                          int nb_norm, int* idx, int epoch, int br, int n,
                                                          unsigned long long sseed, CglOpPack pk) {
  cgl_round_prologue_at(blockIdx.x, gridDim.x, a, z, nz, zseed, nb_norm, idx, epoch, br, n, sseed, pk);
}
#endif

// The round prologue fused with G's first GEMM (K_GEMM_PRO, fuse_prologue): workgroups [0, gemm_wgs) run
// the GEMM, each drawing its own rows of z first (a_gen); the rest run the prologue's other blocks
// (round scalars, real-batch sampler, operand packing), which nothing in this launch reads.
}  // namespace

template <int TM, int TN>
__global__ __launch_bounds__(CGL_GEMM_THREADS) void cgl_gemm_pro(const CglGemmDesc* __restrict__ descs, int gemm_wgs,
                                                                const int* __restrict__ pf, int pf_lines, CglBeginArgs a, float* z, long nz,
                                                                unsigned long long zseed, int* idx, int epoch, int br,
                                                                int n, unsigned long long sseed, CglOpPack pk) {
  extern __shared__ float cgl_dyn_lds[];
  __shared__ int s_flag[1];
  __shared__ double s_bnd[4 * TN * 32 * 2];
  const int bid = blockIdx.x;
  if (bid >= gemm_wgs) {
    cgl_round_prologue_at(bid - gemm_wgs, (int)gridDim.x - gemm_wgs, a, z, nz, zseed, 0, idx, epoch, br, n, sseed, pk);
    return;
  }
  int pfv = 0;     // the next GEMM launch's descriptors into every XCD's L2 (as cgl_gemm_f32)
  if (bid < 8 && (int)threadIdx.x < pf_lines) pfv = pf[threadIdx.x * 32];
  const CglGemmDesc* __restrict__ d = descs;
  if (d->layout != 0) return;     // planner: an NT problem (A = z rows)
  if (d->a_vec && d->b_vec)
    cgl_gemm_body<0, 1, TM, TN, false, CGL_DTYPE_F32, 0>(d, bid, cgl_dyn_lds, s_flag, s_bnd);
  else
    cgl_gemm_body<0, 0, TM, TN, false, CGL_DTYPE_F32, 0>(d, bid, cgl_dyn_lds, s_flag, s_bnd);
  asm volatile("" ::"v"(pfv));
}
