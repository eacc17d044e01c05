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
                                                                CglBeginArgs a, float* z, long nz,
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
  const CglGemmDesc* __restrict__ d = descs;
  if (d->layout != 0) return;     // planner: an NT problem (A = z rows)
  if (d->a_vec && d->b_vec)
    cgl_gemm_body<0, 1, TM, TN, false, CGL_DTYPE_F32, 0>(d, bid, cgl_dyn_lds, s_flag, s_bnd);
  else
    cgl_gemm_body<0, 0, TM, TN, false, CGL_DTYPE_F32, 0>(d, bid, cgl_dyn_lds, s_flag, s_bnd);
}
