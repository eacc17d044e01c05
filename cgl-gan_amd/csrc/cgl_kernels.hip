// Non-GEMM kernels of the MLP GAN step (gfx950).
//
//  cgl_head_loss   D output layer (2 logits or 1 Sigmoid unit) + CrossEntropy / BCE loss, its
//                  backward into the last hidden layer, and the batch-mean loss reduced by the
//                  last-arriving workgroup (reference: nn.Linear(256,2) model/mnist_model.py:81,
//                  nn.CrossEntropyLoss capgan.py:311, nn.BCELoss CGLGAN/2DMG/main.py:336).
//  cgl_bn_bwd      BatchNorm1d(eps=0.8) train-mode backward fused with the LeakyReLU' mask of its
//                  output (model/mnist_model.py:13-14; autograd in Server.train capgan.py:258).
//  cgl_adam        flat multi-tensor Adam, op order of torch 2.10 _single_tensor_adam
//                  (optim.Adam(lr=2e-4, betas=(0.5, 0.999)) capgan.py:158,312), plus the scalar
//                  tail of the round (lambda SGD capgan.py:140-141,259; F_max :249).
//  cgl_begin_at    per-round Adam bias corrections (device-side, graph-replayable).
//  cgl_normal      Philox4x32-10 + Box-Muller N(0,1) for z (capgan.py:216,219).
//  cgl_alpha_scale lambda-weighting of gathered worker losses (capgan.py:247-248,
//                  mixed-gan.py:276, MDGAN/MNIST/mdgan.py:203, CGLGAN/2DMG/main.py:261-264) and the
//                  scaling of this worker's gradient contribution before the RCCL all-reduce.
#include "cgl_internal.h"

// ------------------------------------------------------------------------------------------
// wave-level sum
__device__ __forceinline__ float cgl_wave_sum(float x) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

// The batch-mean losses from the nwg per-workgroup partials (every thread of the calling workgroup loads
// them at once, one round trip; thread 0 sums them in a fixed order, in double) -- run by the head's last
// arriving workgroup, or by the finisher workgroup of the next GEMM launch when the head is deferred.
__device__ void cgl_head_finish(const CglHeadDesc* __restrict__ hd, int nwg, float* s_part) {
  const int M = hd->M;
  // every thread loads partials at once (one round trip), thread 0 sums them in a fixed order
  const int np = 2 * nwg;
  for (int i = threadIdx.x; i < np; i += 256)
    s_part[i] = __hip_atomic_load((CGL_GLOBAL float*)(hd->part + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (threadIdx.x == 0) {
    double s0 = 0.0, s1 = 0.0;
    for (int q = 0; q < nwg; ++q) {
      s0 += (double)s_part[2 * q];
      s1 += (double)s_part[2 * q + 1];
    }
    const int n0s = min(hd->split, M), n1 = M - n0s;
    const int n0 = hd->n0_dev ? min(gldi(hd->n0_dev), n0s) : n0s;
    const float l0 = n0 > 0 ? (float)(s0 / n0) : (hd->combine_in0 ? gld(hd->combine_in0) : 0.f);
    const float l1 = n1 > 0 ? (float)(s1 / n1) : 0.f;
    if (hd->loss_out0 && n0 > 0) gst(hd->loss_out0, l0);
    if (hd->loss_out2 && n0 > 0) gst(hd->loss_out2, l0);
    if (hd->loss_out1 && n1 > 0) gst(hd->loss_out1, l1);
    if (hd->combine_out) gst(hd->combine_out, (l0 + l1) * hd->combine);
  }
}

#define CGL_HEAD_MAXQ 4   // float4 per lane kept in registers: F <= 1024
#ifndef CGL_GEMM_PART_TU   // (the GEMM-instantiation translation units compile only device functions)
__device__ __forceinline__ void cgl_head_loss_body(const CglHeadDesc* __restrict__ hd, int bid, int nwg) {
  // Each wave owns rows r0 + wave + 4 i; a row is a dot product of F features (F % 4 == 0)
  // over 16-byte loads held in registers, a 64-lane reduction, the loss and its gradient, then
  // the gradient into the last hidden layer (dlogits . W) * LeakyReLU'(P) from the same
  // registers.  The batch-mean losses are reduced by the last workgroup to arrive.
  __shared__ float s_loss[4][2];
  __shared__ int s_last;
  __shared__ float s_part[2 * 1024];
  const int M = hd->M, F = hd->F, C = hd->C;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int n0 = hd->n0_dev ? gldi(hd->n0_dev) : hd->split;
  const float wr0 = hd->n0_dev ? hd->combine / (float)n0 : hd->w0;   // real-segment dlogit weight
  const float lsc = hd->scale_dev ? gld(hd->scale_dev) : 1.f;         // dynamic loss scale (power of 2)
  const int lane = threadIdx.x & 63;
  const int r0 = bid * hd->rows_per_wg;
  const int r1 = min(r0 + hd->rows_per_wg, M);
  const float* __restrict__ Pb = hd->P;
  const float* __restrict__ W = hd->W;
  const int F4 = F >> 2;
  const float b0 = gld(hd->b), b1 = C == 2 ? gld(hd->b + 1) : 0.f;
  // W rows (same for every row of the batch)
  f32x4 w0[CGL_HEAD_MAXQ], w1[CGL_HEAD_MAXQ];
#pragma unroll
  for (int u = 0; u < CGL_HEAD_MAXQ; ++u) {
    const int q = min(lane + 64 * u, F4 - 1);
    w0[u] = *(gcf4p)(W + 4 * q);
    w1[u] = C == 2 ? *(gcf4p)(W + F + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  float lsum[2] = {0.f, 0.f};
  for (int r = r0 + wave; r < r1; r += 4) {
    const float* p = Pb + (long)r * hd->ldp;
    f32x4 pv[CGL_HEAD_MAXQ];
#pragma unroll
    for (int u = 0; u < CGL_HEAD_MAXQ; ++u) pv[u] = *(gcf4p)(p + 4 * min(lane + 64 * u, F4 - 1));
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int u = 0; u < CGL_HEAD_MAXQ; ++u) {
      if (lane + 64 * u < F4) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s0 = fmaf(pv[u][e], w0[u][e], s0);
          s1 = fmaf(pv[u][e], w1[u][e], s1);
        }
      }
    }
    float z[2];
    z[0] = cgl_wave_sum(s0) + b0;
    z[1] = C == 2 ? cgl_wave_sum(s1) + b1 : 0.f;
    const int seg = r < hd->split ? 0 : 1;
    const int t = seg ? hd->t1 : hd->t0;
    // a device-sized real segment (the sampler's short batch): rows past n0 carry nothing
    const bool dead = seg == 0 && r >= n0;
    const float wgt = (dead ? 0.f : seg ? hd->w1 : wr0) * lsc;
    float dl[2];
    float lossv;
    if (hd->loss == 0) {
      // log_softmax over the 2 logits + NLL (torch: x - max - log(sum(exp(x - max))))
      const float mx = fmaxf(z[0], z[1]);
      const float se = expf(z[0] - mx) + expf(z[1] - mx);
      const float lse = logf(se);
      const float o0 = z[0] - mx - lse, o1 = z[1] - mx - lse;
      lossv = -(t == 0 ? o0 : o1);
      // NLL backward (-w at target) through log_softmax backward: g - exp(out) * sum(g)
      dl[0] = (t == 0 ? -wgt : 0.f) + expf(o0) * wgt;
      dl[1] = (t == 1 ? -wgt : 0.f) + expf(o1) * wgt;
    } else {
      // Sigmoid + BCELoss (log clamped at -100, EPSILON 1e-12 in the backward)
      const float pr = 1.f / (1.f + expf(-z[0]));
      const float y = (float)t;
      const float lp = fmaxf(logf(pr), -100.f), l1p = fmaxf(logf(1.f - pr), -100.f);
      lossv = -(y * lp + (1.f - y) * l1p);
      const float gp = wgt * (pr - y) / fmaxf((1.f - pr) * pr, 1e-12f);
      dl[0] = gp * (1.f - pr) * pr;
      dl[1] = 0.f;
    }
    if (!dead) lsum[seg] += lossv;
    if (hd->dlogits && lane < C) gst(hd->dlogits + (long)r * C + lane, dl[lane]);
    if (hd->dP) {
      float* dp = hd->dP + (long)r * hd->lddp;
      const float sl = hd->slope;
#pragma unroll
      for (int u = 0; u < CGL_HEAD_MAXQ; ++u) {
        const int q = lane + 64 * u;
        if (q < F4) {
          f32x4 g = dl[0] * w0[u];
          if (C == 2) {
            g[0] = fmaf(dl[1], w1[u][0], g[0]);
            g[1] = fmaf(dl[1], w1[u][1], g[1]);
            g[2] = fmaf(dl[1], w1[u][2], g[2]);
            g[3] = fmaf(dl[1], w1[u][3], g[3]);
          }
          f32x4 o;
          for (int e = 0; e < 4; ++e) o[e] = pv[u][e] > 0.f ? g[e] : g[e] * sl;
          *(gf4p)(dp + 4 * q) = o;
        }
      }
    }
  }
  if (lane == 0) {
    s_loss[wave][0] = lsum[0];
    s_loss[wave][1] = lsum[1];
  }
  __syncthreads();
  if (hd->deferred) {   // the next launch's finisher workgroup reduces the partials (kernel boundary = visibility)
    if (threadIdx.x == 0) {
      float a = 0.f, b = 0.f;
      for (int q = 0; q < 4; ++q) {
        a += s_loss[q][0];
        b += s_loss[q][1];
      }
      gst(hd->part + bid * 2 + 0, a);
      gst(hd->part + bid * 2 + 1, b);
    }
    return;
  }
  if (threadIdx.x == 0) {
    float a = 0.f, b = 0.f;
    for (int q = 0; q < 4; ++q) {
      a += s_loss[q][0];
      b += s_loss[q][1];
    }
    // last-arriver reduction: partials are published with agent-coherent (sc1) stores and
    // complete before the ticket is taken; the last workgroup reads them back coherently
    __hip_atomic_store((CGL_GLOBAL float*)(hd->part + bid * 2 + 0), a, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((CGL_GLOBAL float*)(hd->part + bid * 2 + 1), b, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned int ticket =
        __hip_atomic_fetch_add(hd->counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (ticket == nwg - 1);
  }
  __syncthreads();
  if (!s_last) return;
  cgl_head_finish(hd, nwg, s_part);
  if (threadIdx.x == 0) __hip_atomic_store(hd->counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
#endif   // CGL_GEMM_PART_TU

// (cgl_bn_stats: cgl_gemm.hip, shared with the GEMMs that fold the BatchNorm into their loads)

// BatchNorm1d(train) + LeakyReLU of one G layer's [mtot][F] output, torch's arithmetic:
//   invstd = 1 / sqrt(var_biased + eps),  scale = invstd * gamma,  shift = beta - mean * scale,
//   act = leaky(fma(y, scale, shift))
// per forward call (group of gr rows).  A workgroup owns 64 features x CGL_BNA_ROWS rows; its
// first 64 x ngroups threads combine the producer partials of its features (one memory round
// trip), the row-block-0 workgroups also write the saved mean / invstd for the backward pass and
// update the running statistics (momentum, unbiased variance) group by group in the order of the
// reference's forward calls (Xd then Xg, capgan.py:215-220).
#define CGL_BNA_ROWS 32
#ifndef CGL_GEMM_PART_TU   // (the GEMM-instantiation translation units compile only device functions)
__device__ __forceinline__ void cgl_bn_apply_body(const CglBnApplyDesc* __restrict__ ad, int bx, int by) {
  __shared__ float s_sc[2][64], s_sh[2][64];
  __shared__ double s_mean[2][64], s_m2[2][64];
  __shared__ int s_n[2];
  const CglBnFwd& bn = ad->bn;
  const int F = ad->F, mtot = bn.mtot;
  const int ngroups = (mtot + bn.gr - 1) / bn.gr;   // <= 2
  const int tid = threadIdx.x, fl = tid & 63, rl = tid >> 6;
  const int f0 = bx * 64, r0 = by * CGL_BNA_ROWS;
  const int f = f0 + fl, fc = min(f, F - 1);
  // this thread's rows, loaded before the statistics are ready
  constexpr int RPT = CGL_BNA_ROWS / 4;
  float y[RPT];
#pragma unroll
  for (int i = 0; i < RPT; ++i) y[i] = gld(ad->Y + (long)min(r0 + rl + 4 * i, mtot - 1) * ad->ld_y + fc);
  // gamma / beta and the running statistics are issued with the rows, ahead of the partials' combine:
  // loaded after it they cost one more dependent memory round trip each (unconditional loads from
  // valid addresses: a predicated load compiles to a branch with a full vmcnt(0) drain)
  const float gam = gld(bn.gamma + fc), bet = gld(bn.beta + fc);
  const float rm0 = gld(bn.run_mean ? bn.run_mean + fc : bn.gamma + fc);
  const float rv0 = gld(bn.run_var ? bn.run_var + fc : bn.gamma + fc);
  if (tid < 64 * ngroups) {
    const int g = tid >> 6;
    const int k[1] = {f < F ? f : -1};
    double mean[1], m2[1];
    int n;
    cgl_bn_stats<1>(bn, F, k, g, mean, m2, n);
    const double invstd = 1.0 / sqrt(m2[0] / n + bn.eps);
    const float sc = (float)invstd * gam;
    s_sc[g][fl] = sc;
    s_sh[g][fl] = bet - (float)mean[0] * sc;
    s_mean[g][fl] = mean[0];
    s_m2[g][fl] = m2[0];
    if (fl == 0) s_n[g] = n;
    if (by == 0 && f < F && bn.save_mean) {
      gst(bn.save_mean + (long)g * F + f, (float)mean[0]);
      gst(bn.save_invstd + (long)g * F + f, (float)invstd);
    }
  }
  __syncthreads();
  if (by == 0 && bn.run_mean && tid < 64 && f < F) {
    const double mom = bn.momentum;
    float rm = rm0, rv = rv0;
    for (int g = 0; g < ngroups; ++g) {
      rm = (float)(mom * s_mean[g][fl] + (1.0 - mom) * (double)rm);
      rv = (float)(mom * (s_m2[g][fl] / (s_n[g] - 1)) + (1.0 - mom) * (double)rv);
    }
    gst(bn.run_mean + f, rm);
    gst(bn.run_var + f, rv);
  }
  if (f >= F) return;
  const float sl = bn.slope;
  const int kc = (F + 15) >> 4;
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int r = r0 + rl + 4 * i;
    if (r < mtot) {
      const int g = r >= bn.gr ? 1 : 0;
      const float x = fmaf(y[i], s_sc[g][fl], s_sh[g][fl]);
      const float a = x > 0.f ? x : x * sl;
      gst(ad->act + (long)r * ad->ld_act + f, a);
      if (ad->act_pk) gst(ad->act_pk + cgl_pk_off(r, f, kc), a);   // the next GEMM's packed A operand
    }
  }
}
#endif   // CGL_GEMM_PART_TU

// ------------------------------------------------------------------------------------------
// BatchNorm1d backward (train) + LeakyReLU' mask.  One workgroup owns 32 features and all M
// rows, so the per-feature reductions stay inside the workgroup (fixed order, double accum):
//   dy = dA * leaky'(post),  S = sum dy,  D = sum (y - mean) dy,
//   dZ = (dy - S/M - (y - mean) D invstd^2 / M) invstd gamma,  dgamma = D invstd,  dbeta = S
// (torch's batch_norm_backward, train mode).  With M <= 8 * CGL_BNB_RPT every thread keeps its
// rows in registers: all loads are issued at once (one memory round trip) and the second pass
// reuses them; larger M streams the rows twice.
#define CGL_BNB_RPT 32
// dgamma / dbeta of feature f, plus the loss-scaling overflow check of those two gradients
__device__ __forceinline__ void cgl_bnb_store_gb(const CglBnBwdDesc* __restrict__ bd, int f, float dg, float db) {
  gst(bd->g_gamma + f, dg);
  gst(bd->g_beta + f, db);
  if (bd->inf_flag && !(isfinite(dg) && isfinite(db))) atomicOr(bd->inf_flag, 1u);
}
// FPW features per workgroup (32: the original layout; 16 / 8 / 4 give 2x / 4x / 8x the workgroups for the narrow
// layers, each thread then owning fewer rows): NRG = 256 / FPW row groups, rows of a group in registers.
template <int FPW>
__device__ __forceinline__ void cgl_bn_bwd_body(const CglBnBwdDesc* __restrict__ bd) {
  constexpr int NRG = 256 / FPW, RPT = 256 / NRG;   // register path: M <= NRG * RPT = 256
  __shared__ double s_a[NRG][FPW], s_b[NRG][FPW];
  const int M = bd->M, F = bd->F;
  const int fl = threadIdx.x % FPW, rg = threadIdx.x / FPW;
  // XCD-contiguous feature slices: workgroup b runs on XCD b % 8, so give each XCD a contiguous range of
  // slices -- the 128 / (4 FPW) slices that share a row's 128-byte lines then fetch (and write) them through
  // one L2 instead of up to four (FPW = 8: 4x the dA / post / Y fetch, profiles/r04_traffic.json)
  int blk = blockIdx.x;
  if (gridDim.x >= 16) {
    const int nb = gridDim.x, xcd = blk & 7, pos = blk >> 3, q = nb >> 3, rr = nb & 7;
    blk = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + pos;
  }
  const int f = blk * FPW + fl;
  const bool fok = f < F;
  const int fc = min(f, F - 1);
  const float sl = bd->slope;
  const float mean = gld(bd->mean + fc);
  const float invstd = gld(bd->invstd + fc);
  const float w = gld(bd->gamma + fc);
  const float* dA = bd->dA + fc;
  const bool post_on = bd->post != nullptr;
  const float* post = post_on ? bd->post + fc : bd->Y + fc;   // (any valid address when unused)
  const float* Y = bd->Y + fc;
  const long lda = bd->ld_da, ldp = bd->ld_post, ldy = bd->ld_y;
  float* dZ = bd->dZ + fc;
  const long ldz = bd->ld_dz;
  const int kcz = (F + 15) >> 4;
  double sum = 0.0, dotp = 0.0;
  if (M <= NRG * RPT) {
    float dy[RPT], yc[RPT];
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
      const int r = min(rg + NRG * j, M - 1);
      // unconditional load (post aliases Y when unused), select after: a predicated load compiles
      // to a branch with a full vmcnt(0) drain per row
      const float da = gld(dA + r * lda), pr = gld(post + r * ldp), y = gld(Y + r * ldy);
      const float po = post_on ? pr : 1.f;
      dy[j] = po > 0.f ? da : da * sl;
      yc[j] = y - mean;
    }
#pragma unroll
    for (int j = 0; j < RPT; ++j) {
      if (rg + NRG * j < M) {
        sum += (double)dy[j];
        dotp += (double)(yc[j] * dy[j]);
      }
    }
    s_a[rg][fl] = sum;
    s_b[rg][fl] = dotp;
    __syncthreads();
    double S = 0.0, D = 0.0;
    for (int q = 0; q < NRG; ++q) {
      S += s_a[q][fl];
      D += s_b[q][fl];
    }
    const float k = (float)D * invstd * invstd / M;
    const float gmean = (float)(S / M);
    if (fok) {
#pragma unroll
      for (int j = 0; j < RPT; ++j) {
        const int r = rg + NRG * j;
        if (r < M) {
          const float z = (dy[j] - gmean - yc[j] * k) * invstd * w;
          gst(dZ + r * ldz, z);
          if (bd->dZ_pk) gst(bd->dZ_pk + cgl_pk_off(r, f, kcz), z);   // the input-gradient GEMM's packed A
        }
      }
      if (rg == 0) cgl_bnb_store_gb(bd, f, (float)(D * (double)invstd), (float)S);
    }
    return;
  }
  for (int r0 = rg; r0 < M; r0 += 8 * NRG) {
    float da[8], po[8], y[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int r = min(r0 + NRG * j, M - 1);
      da[j] = gld(dA + r * lda);
      po[j] = gld(post + r * ldp);
      y[j] = gld(Y + r * ldy);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (r0 + NRG * j < M) {
        const float dy = (!post_on || po[j] > 0.f) ? da[j] : da[j] * sl;
        sum += (double)dy;
        dotp += (double)((y[j] - mean) * dy);
      }
    }
  }
  s_a[rg][fl] = sum;
  s_b[rg][fl] = dotp;
  __syncthreads();
  double S = 0.0, D = 0.0;
  for (int q = 0; q < NRG; ++q) {
    S += s_a[q][fl];
    D += s_b[q][fl];
  }
  if (!fok) return;
  const float k = (float)D * invstd * invstd / M;
  const float gmean = (float)(S / M);
  for (int r0 = rg; r0 < M; r0 += 8 * NRG) {
    float da[8], po[8], y[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int r = min(r0 + NRG * j, M - 1);
      da[j] = gld(dA + r * lda);
      po[j] = gld(post + r * ldp);
      y[j] = gld(Y + r * ldy);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int r = r0 + NRG * j;
      if (r < M) {
        const float dy = (!post_on || po[j] > 0.f) ? da[j] : da[j] * sl;
        const float gi = (y[j] - mean) * k;
        const float z = (dy - gmean - gi) * invstd * w;
        gst(dZ + r * ldz, z);
        if (bd->dZ_pk) gst(bd->dZ_pk + cgl_pk_off(r, f, kcz), z);
      }
    }
  }
  if (rg == 0) cgl_bnb_store_gb(bd, f, (float)(D * (double)invstd), (float)S);
}

#ifndef CGL_GEMM_PART_TU   // (the GEMM-instantiation translation units compile only device functions)
// The round's small kernels take their descriptor BY VALUE (the kernel arguments): its fields arrive with the
// kernarg fetch instead of one more dependent scalar round trip to a descriptor in memory (tools/launch_probe.hip:
// ~0.16 us per dependent scalar load).  The workspace copies stay (the deferred head reduction reads its head's).
__global__ __launch_bounds__(256) void cgl_head_loss(const CglHeadDesc d) {
  cgl_head_loss_body(&d, blockIdx.x, gridDim.x);
}
__global__ __launch_bounds__(256) void cgl_bn_apply(const CglBnApplyDesc d) {
  cgl_bn_apply_body(&d, blockIdx.x, blockIdx.y);
}
__global__ __launch_bounds__(256) void cgl_bn_bwd(const CglBnBwdDesc d) { cgl_bn_bwd_body<32>(&d); }
__global__ __launch_bounds__(256) void cgl_bn_bwd16(const CglBnBwdDesc d) { cgl_bn_bwd_body<16>(&d); }
__global__ __launch_bounds__(256) void cgl_bn_bwd8(const CglBnBwdDesc d) { cgl_bn_bwd_body<8>(&d); }
__global__ __launch_bounds__(256) void cgl_bn_bwd4(const CglBnBwdDesc d) { cgl_bn_bwd_body<4>(&d); }
// the single-op entry point (cgl_bn1d_bwd): the descriptor travels in the kernel arguments
__global__ __launch_bounds__(256) void cgl_bn_bwd_arg(const CglBnBwdDesc d) { cgl_bn_bwd_body<32>(&d); }
#endif   // CGL_GEMM_PART_TU
// ------------------------------------------------------------------------------------------
// Standalone BatchNorm1d (+ LeakyReLU) forward, train or eval, for the nn.Module path.  One
// workgroup owns 32 features x all M rows (8 row groups): column sums in double, fixed order;
// rows stay in registers when M <= 8 * CGL_BNB_RPT (one memory round trip), else are streamed.
__device__ __forceinline__ void cgl_bn1d_apply_row(const CglBn1dDesc* bd, int r, int f, float x, float sc, float sh) {
  float y = fmaf(x, sc, sh);
  if (bd->act == CGL_EPI_ACT_LEAKY) y = y > 0.f ? y : y * bd->slope;
  gst(bd->Y + (long)r * bd->F + f, y);
}

#ifndef CGL_GEMM_PART_TU   // (the GEMM-instantiation translation units compile only device functions)
__global__ __launch_bounds__(256) void cgl_bn1d_fwd_k(const CglBn1dDesc d) {   // descriptor in the kernel arguments
  const CglBn1dDesc* __restrict__ bd = &d;
  __shared__ double s_a[8][32];
  __shared__ float s_sc[32], s_sh[32];
  const int M = bd->M, F = bd->F;
  const int fl = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int f = blockIdx.x * 32 + fl;
  const bool fok = f < F;
  const int fc = min(f, F - 1);
  const float* X = bd->X + fc;
  const long ldx = bd->ldx;
  const bool regs = M <= 8 * CGL_BNB_RPT;
  float xv[CGL_BNB_RPT];
  if (regs) {
#pragma unroll
    for (int j = 0; j < CGL_BNB_RPT; ++j) xv[j] = gld(X + (long)min(rg + 8 * j, M - 1) * ldx);
  }
  if (bd->train) {
    double sum = 0.0;
    if (regs) {
#pragma unroll
      for (int j = 0; j < CGL_BNB_RPT; ++j)
        if (rg + 8 * j < M) sum += (double)xv[j];
    } else {
      for (int r = rg; r < M; r += 8) sum += (double)gld(X + (long)r * ldx);
    }
    s_a[rg][fl] = sum;
    __syncthreads();
    double S = 0.0;
    for (int q = 0; q < 8; ++q) S += s_a[q][fl];
    const double mean = S / M;
    __syncthreads();
    double q2 = 0.0;
    if (regs) {
#pragma unroll
      for (int j = 0; j < CGL_BNB_RPT; ++j)
        if (rg + 8 * j < M) {
          const double dd = (double)xv[j] - mean;
          q2 += dd * dd;
        }
    } else {
      for (int r = rg; r < M; r += 8) {
        const double dd = (double)gld(X + (long)r * ldx) - mean;
        q2 += dd * dd;
      }
    }
    s_a[rg][fl] = q2;
    __syncthreads();
    if (rg == 0) {
      double Q = 0.0;
      for (int q = 0; q < 8; ++q) Q += s_a[q][fl];
      const double var = Q / M;
      const double invstd = 1.0 / sqrt(var + bd->eps);
      const float sc = (float)invstd * gld(bd->gamma + fc);
      s_sc[fl] = sc;
      s_sh[fl] = gld(bd->beta + fc) - (float)mean * sc;
      if (fok) {
        if (bd->save_mean) {
          gst(bd->save_mean + f, (float)mean);
          gst(bd->save_invstd + f, (float)invstd);
        }
        if (bd->run_mean) {
          const double mom = bd->momentum;
          gst(bd->run_mean + f, (float)(mom * mean + (1.0 - mom) * (double)gld(bd->run_mean + f)));
          const double unb = M > 1 ? Q / (M - 1) : var;
          gst(bd->run_var + f, (float)(mom * unb + (1.0 - mom) * (double)gld(bd->run_var + f)));
        }
      }
    }
  } else if (rg == 0) {
    const double invstd = 1.0 / sqrt((double)gld(bd->run_var + fc) + bd->eps);
    const float sc = (float)invstd * gld(bd->gamma + fc);
    s_sc[fl] = sc;
    s_sh[fl] = gld(bd->beta + fc) - gld(bd->run_mean + fc) * sc;
  }
  __syncthreads();
  if (!fok) return;
  const float sc = s_sc[fl], sh = s_sh[fl];
  if (regs) {
#pragma unroll
    for (int j = 0; j < CGL_BNB_RPT; ++j)
      if (rg + 8 * j < M) cgl_bn1d_apply_row(bd, rg + 8 * j, f, xv[j], sc, sh);
  } else {
    for (int r = rg; r < M; r += 8) cgl_bn1d_apply_row(bd, r, f, gld(X + (long)r * ldx), sc, sh);
  }
}

// elementwise activation forward / backward (act: 1 LeakyReLU, 2 Tanh, 3 Sigmoid)
__global__ __launch_bounds__(256) void cgl_act_fwd_k(const float* X, long n, int act, float slope, float* Y) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float x = gld(X + i);
    float y = x;
    if (act == CGL_EPI_ACT_LEAKY) y = x > 0.f ? x : x * slope;
    else if (act == CGL_EPI_ACT_TANH) y = cgl_tanh(x);
    else if (act == CGL_EPI_ACT_SIGMOID) y = 1.f / (1.f + expf(-x));
    gst(Y + i, y);
  }
}

__global__ __launch_bounds__(256) void cgl_act_bwd_k(const float* dY, const float* Y, long n, int act, float slope,
                                                     float* dX) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float g = gld(dY + i), y = gld(Y + i);
    float d = g;
    if (act == CGL_EPI_ACT_LEAKY) d = y > 0.f ? g : g * slope;
    else if (act == CGL_EPI_ACT_TANH) d = cgl_dtanh(g, y);
    else if (act == CGL_EPI_ACT_SIGMOID) d = g * (y * (1.f - y));
    gst(dX + i, d);
  }
}

#endif   // CGL_GEMM_PART_TU
// ------------------------------------------------------------------------------------------
struct CglAdamArgs {
  float* p; float* g; float* m; float* v;
  long n;
  const float* step_size;   // device scalars (CglStepState fields)
  const float* bc2sqrt;
  float b2, w1, w2, eps;   // w1 = (float)(1 - beta1), w2 = (float)(1 - beta2) computed in double
  // dynamic loss scaling (null: off): the gradients carry *scale; they are unscaled in place (torch's
  // GradScaler.unscale_: g * fp32(1 / scale), exact for a power of two) and the step is skipped when
  // *found (a non-finite weight gradient of this model this round) is set
  const float* scale;
  const unsigned int* found;
  // step_size / bc2sqrt == null: the values themselves, passed in the kernel arguments (cgl_adam_step: no
  // upload, so the single-op Adam needs no host synchronisation and can be captured)
  float step_size_v, bc2sqrt_v;
  // z one round ahead (the G Adam launch, plan z_ahead): blocks [zblk0, grid) draw the next round's z into znext
  // (nz floats, Philox stream 0 of seed zseed, counter = the round in progress + 1: the draw the next round's
  // prologue made before), while the other blocks update the parameters
  float* znext;
  long nz;
  unsigned long long zseed;
  int zblk0;
};
__device__ __forceinline__ bool cgl_adam_zblock(const CglAdamArgs& a, const CglStepState* st) {
  if (!a.znext || (int)blockIdx.x < a.zblk0) return false;
  cgl_normal_at((long)(blockIdx.x - a.zblk0) * 256 + threadIdx.x, a.znext, a.nz, a.zseed,
                (uint32_t)(st->cur_round + 1), 0);
  return true;
}



// alpha_i for every worker from the gathered losses (the reference's Server.train weighting).

// Scalar tail of Server.train: F_max and the lambda update (after every parameter read of this
// round, before the next round's prologue).  Written without per-worker local arrays (alpha_i is
// recomputed per worker, O(N^2) for N <= 64 in one thread) so that the kernels it is inlined into
// (cgl_adam, the GEMM launch carrying the folded Adam) need no scratch memory; the arithmetic and
// its order are those of cgl_weights / cgl_softmax_at.
__device__ __forceinline__ float cgl_tail_loss(const CglStepState* st, int q) {
  return st->n_workers == 1 ? st->g_loss_parts[0] : st->losses[q];
}
// softmax(lam * l)_i
__device__ float cgl_tail_sm1(const CglStepState* st, float lam, int i) {
  const int N = st->n_workers;
  float mx = lam * cgl_tail_loss(st, 0);
  for (int q = 1; q < N; ++q) mx = fmaxf(mx, lam * cgl_tail_loss(st, q));
  float s = 0.f;
  for (int q = 0; q < N; ++q) s += expf(lam * cgl_tail_loss(st, q) - mx);
  return expf(lam * cgl_tail_loss(st, i) - mx) / s;
}
// the pre-softmax argument of alpha's outer softmax for worker i (modes CAPGAN / MIX_*)
__device__ float cgl_tail_arg(const CglStepState* st, int mode, float lam, int i) {
  if (mode == CGL_W_MIX_SINGLE) return st->beta[i] * lam * cgl_tail_loss(st, i);
  if (mode == CGL_W_CAPGAN) return cgl_tail_sm1(st, lam, i) * st->beta[i];
  return st->beta[i] * cgl_tail_sm1(st, lam, i);   // CGL_W_MIX_DOUBLE
}
__device__ float cgl_tail_alpha(const CglStepState* st, int mode, float lam, int i) {
  const int N = st->n_workers;
  float mx = cgl_tail_arg(st, mode, lam, 0);
  for (int q = 1; q < N; ++q) mx = fmaxf(mx, cgl_tail_arg(st, mode, lam, q));
  float s = 0.f;
  for (int q = 0; q < N; ++q) s += expf(cgl_tail_arg(st, mode, lam, q) - mx);
  return expf(cgl_tail_arg(st, mode, lam, i) - mx) / s;
}
__device__ void cgl_round_tail(CglStepState* st) {
  const int N = st->n_workers;
  const float lam = st->lambda;
  const int mode = st->weighting;
  if (mode == CGL_W_MEAN) {
    float s = 0.f;
    for (int q = 0; q < N; ++q) s += cgl_tail_loss(st, q);
    st->F = s / N;
  } else if (mode == CGL_W_CGLGAN) {
    float fb = 0.f, fg = 0.f, g1 = 0.f, g2 = 0.f;
    for (int q = 0; q < N; ++q) {
      const float lq = cgl_tail_loss(st, q);
      fb += st->beta[q] * lq;
      fg += cgl_tail_sm1(st, lam, q) * lq;
    }
    st->F = (fb + fg) / 2.f;
    for (int q = 0; q < N; ++q) {
      const float lq = cgl_tail_loss(st, q), gm = cgl_tail_sm1(st, lam, q);
      g1 += lq * lq * gm;
      g2 += lq * gm * fg;
    }
    st->lambda = lam + 10.f * (g1 - g2);
  } else {
    float s = 0.f;
    for (int q = 0; q < N; ++q) s += cgl_tail_alpha(st, mode, lam, q) * cgl_tail_loss(st, q);
    st->F = s - 0.001f * lam;
    // optim.SGD([Lambda], lr=0.1): dF/dLambda = -0.001
    st->lambda = lam + (-0.1f) * (-0.001f);
  }
  st->round = st->round + 1;   // round complete (read by the next round's prologue)
}

__device__ __forceinline__ void cgl_adam_at(const CglAdamArgs& a, CglStepState* st, int tail, long i) {
  const float ss = a.step_size ? gld(a.step_size) : a.step_size_v;
  const float bc = a.bc2sqrt ? gld(a.bc2sqrt) : a.bc2sqrt_v;
  if (a.scale) {
    const float inv = (float)(1.0 / (double)gld(a.scale));
    const bool skip = *(const CGL_GLOBAL unsigned int*)a.found != 0u;
    if (i < a.n) {
      const float g = gld(a.g + i) * inv;
      gst(a.g + i, g);
      if (!skip) {
        float p = gld(a.p + i), m = gld(a.m + i), v = gld(a.v + i);
        cgl_adam_update(p, g, m, v, ss, bc, a.b2, a.w1, a.w2, a.eps);
        gst(a.m + i, m);
        gst(a.v + i, v);
        gst(a.p + i, p);
      }
    }
  } else if (i < a.n) {
    float p = gld(a.p + i), m = gld(a.m + i), v = gld(a.v + i);
    cgl_adam_update(p, gld(a.g + i), m, v, ss, bc, a.b2, a.w1, a.w2, a.eps);
    gst(a.m + i, m);
    gst(a.v + i, v);
    gst(a.p + i, p);
  }
  if (tail && i == 0) {
    cgl_round_tail(st);
    if (a.scale) st->scaler_pending = 1;   // GradScaler.update runs in the next round's prologue
  }
}

#ifndef CGL_GEMM_PART_TU   // (the GEMM-instantiation translation units compile only device functions)
__global__ __launch_bounds__(256) void cgl_adam(CglAdamArgs a, CglStepState* st, int tail) {
  if (cgl_adam_zblock(a, st)) return;
  cgl_adam_at(a, st, tail, (long)blockIdx.x * blockDim.x + threadIdx.x);
}

// The same update four elements per thread with 16-byte loads and stores (n % 4 == 0, 16-byte aligned buffers;
// CglAdamArgs.v4 planned by push_adam): element by element the arithmetic of cgl_adam_at (cgl_adam_update is
// pinned against contraction), so bitwise the scalar launch, on a quarter of the workgroups.
__global__ __launch_bounds__(256) void cgl_adam4(CglAdamArgs a, CglStepState* st, int tail) {
  if (cgl_adam_zblock(a, st)) return;
  const long i4 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const float ss = a.step_size ? gld(a.step_size) : a.step_size_v;
  const float bc = a.bc2sqrt ? gld(a.bc2sqrt) : a.bc2sqrt_v;
  if (i4 < a.n) {
    f32x4 g = *(gcf4p)(a.g + i4);
    bool upd = true;
    if (a.scale) {
      const float inv = (float)(1.0 / (double)gld(a.scale));
      upd = *(const CGL_GLOBAL unsigned int*)a.found == 0u;
#pragma unroll
      for (int e = 0; e < 4; ++e) g[e] = g[e] * inv;
      *(gf4p)(a.g + i4) = g;
    }
    if (upd) {
      f32x4 p = *(gcf4p)(a.p + i4), m = *(gcf4p)(a.m + i4), v = *(gcf4p)(a.v + i4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float pp = p[e], mm = m[e], vv = v[e];
        cgl_adam_update(pp, g[e], mm, vv, ss, bc, a.b2, a.w1, a.w2, a.eps);
        p[e] = pp;
        m[e] = mm;
        v[e] = vv;
      }
      *(gf4p)(a.m + i4) = m;
      *(gf4p)(a.v + i4) = v;
      *(gf4p)(a.p + i4) = p;
    }
  }
  if (tail && i4 == 0) {
    cgl_round_tail(st);
    if (a.scale) st->scaler_pending = 1;
  }
}

// The next round's z from the device round state (cgl_gan_create / _reset / _sync_params): counter st->round + 1,
// the draw that round's prologue would make
__global__ __launch_bounds__(256) void cgl_znext_draw(float* out, long n, unsigned long long seed,
                                                      const CglStepState* st) {
  cgl_normal_at((long)blockIdx.x * 256 + threadIdx.x, out, n, seed, (uint32_t)(st->round + 1), 0);
}
#endif   // CGL_GEMM_PART_TU

// G's first-layer weight gradient fused with the G Adam launch (the round's last two launches as one):
// workgroups [0, gemm_wgs) run the weight-gradient GEMM (ADAM instantiation: each tile applies Adam to
// the parameters it owns from the gradient values it stores), the rest run cgl_adam over every other G
// parameter (`comp`, which does not depend on this GEMM) and the round's scalar tail.  Same arithmetic as
// the two launches, so bitwise the same round.
template <int TM, int TN>
__global__ __launch_bounds__(CGL_GEMM_THREADS) void cgl_gemm_adam(const CglGemmDesc* __restrict__ descs, int ndesc,
                                                                 int gemm_wgs, CglAdamArgs comp, CglStepState* st,
                                                                 int tail) {
  extern __shared__ float cgl_dyn_lds[];
  __shared__ int s_flag[1];
  __shared__ double s_bnd[4 * TN * 32 * 2];
  const int bid = blockIdx.x;
  if (bid >= gemm_wgs) {
    cgl_adam_at(comp, st, tail, (long)(bid - gemm_wgs) * CGL_GEMM_THREADS + threadIdx.x);
    return;
  }
  int di = 0;
  for (int q = 1; q < ndesc; ++q)
    if (bid >= descs[q].wg_begin) di = q;
  const CglGemmDesc* __restrict__ d = descs + di;
  if (d->layout != 2) return;     // planner: the fused weight gradient is a TN problem
  if (d->a_vec && d->b_vec)
    cgl_gemm_body<2, 1, TM, TN, false, CGL_DTYPE_F32, 0, true>(d, bid, cgl_dyn_lds, s_flag, s_bnd);
  else
    cgl_gemm_body<2, 0, TM, TN, false, CGL_DTYPE_F32, 0, true>(d, bid, cgl_dyn_lds, s_flag, s_bnd);
}

// ------------------------------------------------------------------------------------------
struct CglBeginArgs {
  CglStepState* st;
  int epoch;
  double lr_g, lr_d, b1, b2;
  int bn_layers;
  int scaling;           // dynamic loss scaling on (then epoch == 1)
  int growth_interval;
};

// GradScaler.update of the previous round (torch's _amp_update_scale: backoff 0.5 after a skipped step,
// x2 after growth_interval clean ones) and torch's Adam step counts (a skipped step does not count).
__device__ void cgl_scaler_update(const CglBeginArgs& a) {
  CglStepState* st = a.st;
  if (!st->scaler_pending) return;
  for (int m = 0; m < 2; ++m) {
    const bool bad = st->found[m] != 0u;
    st->last_skipped[m] = bad ? 1 : 0;
    if (bad) {
      st->scale[m] *= 0.5f;
      st->growth[m] = 0;
      st->skipped[m] += 1;
    } else {
      st->adam_t[m] += 1;
      const int g = st->growth[m] + 1;
      if (g == a.growth_interval) {
        const float ns = st->scale[m] * 2.f;
        if (isfinite(ns)) st->scale[m] = ns;
        st->growth[m] = 0;
      } else {
        st->growth[m] = g;
      }
    }
    st->found[m] = 0u;
  }
  st->scaler_pending = 0;
}

// Per-round scalars of round r (1-based): Adam bias corrections of the G update and of every
// local D step (torch's step counters: G steps once per round, D `epoch` times), alpha reset,
// BatchNorm num_batches_tracked (two train-mode forward calls per round).  Runs in the round
// prologue; the round counter itself is advanced by the G-Adam tail at the end of the round,
// so that no kernel reads a counter another block of the same launch is writing.
__device__ void cgl_begin_at(const CglBeginArgs& a, int r) {
  CglStepState* st = a.st;
  if (a.scaling) cgl_scaler_update(a);
  {
    // with loss scaling torch's step count is the number of steps taken, not the round
    const double t = a.scaling ? (double)(st->adam_t[1] + 1) : (double)r;
    const double bc1 = 1.0 - pow(a.b1, t);
    const double bc2 = 1.0 - pow(a.b2, t);
    st->g_step_size = (float)(a.lr_g / bc1);
    st->g_bc2sqrt = (float)pow(bc2, 0.5);
  }
  for (int e = 0; e < a.epoch; ++e) {
    const double t = a.scaling ? (double)(st->adam_t[0] + 1) : (double)((r - 1) * a.epoch + e + 1);
    const double bc1 = 1.0 - pow(a.b1, t);
    const double bc2 = 1.0 - pow(a.b2, t);
    st->d_step_size[e] = (float)(a.lr_d / bc1);
    st->d_bc2sqrt[e] = (float)pow(bc2, 0.5);
  }
  st->alpha = 1.f;
  st->bn_batches += 2;
  st->cur_round = r;
}

// ------------------------------------------------------------------------------------------
// Philox4x32-10 counter-based RNG + Box-Muller: out[i] ~ N(0,1), fresh per round.

#ifndef CGL_GEMM_PART_TU   // (the GEMM-instantiation translation units compile only device functions)
__global__ __launch_bounds__(256) void cgl_normal(float* out, long n, unsigned long long seed, int round,
                                                  int stream_id) {
  cgl_normal_at((long)blockIdx.x * blockDim.x + threadIdx.x, out, n, seed, (uint32_t)round, stream_id);
}

// ------------------------------------------------------------------------------------------
// alpha from the gathered losses; scale this worker's gradient buffer by alpha[rank].
__global__ __launch_bounds__(256) void cgl_alpha_scale(CglStepState* st, const float* losses, float* x,
                                                       long n) {
  __shared__ float s_alpha;
  __shared__ float al[CGL_MAX_WORKERS], s_t[2][CGL_MAX_WORKERS];
  if (threadIdx.x == 0) {
    const int N = st->n_workers;
    cgl_weights(st->weighting, N, st->lambda, st->beta, losses, al, s_t[0], s_t[1]);
    s_alpha = al[st->rank];
    if (blockIdx.x == 0) {
      for (int q = 0; q < N; ++q) {
        st->losses[q] = losses[q];
        st->alphas[q] = al[q];
      }
      st->alpha = al[st->rank];
    }
  }
  __syncthreads();
  const float a = s_alpha;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    x[i] *= a;
}

// The gathered exchange (cgl_gan_exchange_mode 1), the head of phase B: slot q of g holds worker q's
// unscaled exchange gradient (n floats) followed by its G loss (word n).  alpha from the N losses exactly as
// cgl_alpha_scale computes it, then x = sum_q alpha_q g_q summed in rank order with every product rounded
// (tot = a_0 g_0; tot += a_1 g_1; ...): bitwise what cgl_alpha_scale on each worker followed by LocalComm's
// rank-ordered sum gives, and the same on every rank (no reduction order left to the collective).
__global__ __launch_bounds__(256) void cgl_alpha_combine(CglStepState* st, const float* __restrict__ g, long slot,
                                                         long n, float* __restrict__ x) {
#pragma clang fp contract(off)
  __shared__ float al[CGL_MAX_WORKERS], s_l[CGL_MAX_WORKERS], s_t[2][CGL_MAX_WORKERS];
  const int N = st->n_workers;
  if ((int)threadIdx.x < N) s_l[threadIdx.x] = g[threadIdx.x * slot + n];
  __syncthreads();
  if (threadIdx.x == 0) {
    cgl_weights(st->weighting, N, st->lambda, st->beta, s_l, al, s_t[0], s_t[1]);
    if (blockIdx.x == 0) {
      for (int q = 0; q < N; ++q) {
        st->losses[q] = s_l[q];
        st->alphas[q] = al[q];
      }
      st->alpha = al[st->rank];
    }
  }
  __syncthreads();
  const long n4 = n >> 2;   // (n % 4 == 0 and 16-byte aligned slots: checked by the planner)
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const f32x4 v0 = *(gcf4p)(g + 4 * i);
    const float a0 = al[0];
    f32x4 t = {a0 * v0[0], a0 * v0[1], a0 * v0[2], a0 * v0[3]};
    for (int q = 1; q < N; ++q) {
      const f32x4 v = *(gcf4p)(g + q * slot + 4 * i);
      const float a = al[q];
      t[0] = t[0] + a * v[0];
      t[1] = t[1] + a * v[1];
      t[2] = t[2] + a * v[2];
      t[3] = t[3] + a * v[3];
    }
    *(gf4p)(x + 4 * i) = t;
  }
}

// y[i] = sum over `parts` contiguous buffers (loopback reduction used by single-device
// multi-worker rehearsal; the multi-GPU path uses RCCL instead)
__global__ __launch_bounds__(256) void cgl_scale_inplace(float* x, long n, float a) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    x[i] *= a;
}
#endif   // CGL_GEMM_PART_TU
