// Internal descriptors shared by the HIP kernels and the host runtime of libcglgan_hip.
// Nothing here crosses the public C-ABI (include/cglgan.h); the runtime builds these
// descriptors once per context, uploads them to device memory and replays them.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/cglgan.h"

#define CGL_WAVE 64
#define CGL_GEMM_THREADS 256
#define CGL_GEMM_KCHUNK 16           // k per MFMA chunk: 8 per lane half (k-permuted)
#define CGL_BN_MAXF 1024             // max features of a G BatchNorm layer

enum { CGL_EPI_ACT_NONE = 0, CGL_EPI_ACT_LEAKY = 1, CGL_EPI_ACT_TANH = 2, CGL_EPI_ACT_SIGMOID = 3 };

// Global-address-space accessors.  Pointers read out of a descriptor in memory are generic to
// the compiler, which then emits flat_* instructions; flat loads return out of order and force
// s_waitcnt vmcnt(0) lgkmcnt(0) at every use.  Every kernel accesses descriptor-borne buffers
// through these so that global_* instructions with counted waits are generated.
#define CGL_GLOBAL __attribute__((address_space(1)))
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef const CGL_GLOBAL float* gcfp;
typedef CGL_GLOBAL float* gfp;
typedef const CGL_GLOBAL f32x4* gcf4p;
typedef CGL_GLOBAL f32x4* gf4p;
__device__ __forceinline__ float gld(const float* p) { return *(gcfp)p; }
#ifdef CGL_GST_WT
// experiment: every plain store write-through at agent scope (no dirty lines left in L2 for the end-of-kernel
// write-back)
__device__ __forceinline__ void gst(float* p, float v) {
  __hip_atomic_store((gfp)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
#else
__device__ __forceinline__ void gst(float* p, float v) { *(gfp)p = v; }
#endif
__device__ __forceinline__ int gldi(const int* p) { return *(const CGL_GLOBAL int*)p; }

// Tanh of the generator output and its derivative.  The derivative 1 - t^2 cancels as |t| -> 1
// (one ulp of t near 0.999 is ~6e-5 of 1 - t^2), so an ulp-level error of a single-precision
// tanh becomes a visible error of every gradient that flows back through the image and of the
// cancelling bias-gradient sum of the output layer.  Both are evaluated in double and rounded
// once: t is then the correctly rounded fp32 tanh (as the CPU reference's) and 1 - t^2 carries
// no cancellation error.  Elementwise on the image only, so the double cost is negligible.
__device__ __forceinline__ float cgl_tanh(float x) { return (float)tanh((double)x); }
__device__ __forceinline__ float cgl_dtanh(float g, float t) {
  const double td = (double)t;
  return (float)((double)g * (1.0 - td * td));
}

// Fragment-packed operand layout P(X; R, K) of the MFMA GEMMs (cgl_gemm.hip): 32-row blocks x 16-k
// chunks x 2 halves x 64 lanes x 4 floats.  Lane l = (r % 32) + 32 lh of a row block holds, for
// chunk c and half h, X[r][16 c + 8 lh + 4 h + e] (e = 0..3) -- the k-permuted 32x32x2 fragment --
// at float ((rb Kc + c) 2 + h) 256 + 4 l + e, so each 16-byte fragment load of a wave reads one
// contiguous 1 KB (8 whole 128-byte lines) instead of 64 pieces of 32 rows.  Padding rows / k
// (past R / K) are never consumed unmasked.
__host__ __device__ inline long cgl_pk_off(int r, int k, int Kc) {
  return ((long)((r >> 5) * Kc + (k >> 4)) * 2 + ((k >> 2) & 1)) * 256 + ((r & 31) + 32 * ((k >> 3) & 1)) * 4 + (k & 3);
}
inline long cgl_pk_floats(int R, int K) { return (long)((R + 31) / 32) * ((K + 15) / 16) * 512; }

// Packing job of the round prologue: dst = P(X; R, K) with X[r][k] = trans ? src[k ld + r] : src[r ld + k]
#define CGL_PACK_MAXJ 12
struct CglOpPackJob {
  const float* src;
  float* dst;
  int R, K, ld, trans;
  int blk_begin;          // first prologue block of this job (one packed float4 per thread)
};
struct CglOpPack {
  int nj, blocks;
  CglOpPackJob j[CGL_PACK_MAXJ];
};

// Row source of a row-major operand whose rows are the non-contiguous index.
// Row r < split comes from p0 (optionally through idx0[idx_off + r]), rows >= split from p1.
struct CglRowSrc {
  const float* p0;
  const float* p1;
  const int* idx0;        // optional gather for segment 0
  const int* idx_off;     // optional device offset added to the gather position
  int split;              // first row of segment 1 (INT32_MAX = single segment)
  int ld;                 // row stride in floats (both segments)
};

// Forward BatchNorm of one G layer.  The producer GEMM wrote per-(row tile, group slot,
// feature) partials {sum, M2}; cgl_bn_apply combines them (fixed order, double) into the
// per-group mean / invstd, applies BatchNorm1d(train) + LeakyReLU, and updates the saved and
// running statistics.
struct CglBnFwd {
  const float* part;      // [ntiles][2][K][2]
  int part_bm;            // producer rows per tile
  int gr;                 // rows per BatchNorm group (one forward call of the reference)
  int mtot;               // total rows in the producer output
  const float* gamma;
  const float* beta;
  double eps, momentum;
  float slope;
  float* run_mean;        // updated group 0 first, then 1 (the reference's call order), may be null
  float* run_var;
  float* save_mean;       // [ngroups][K], may be null
  float* save_invstd;
};

// Backward BatchNorm1d of a GEMM's A operand (a_bn 2): the A values are dy (LeakyReLU'-masked
// gradient w.r.t. the BatchNorm output) stored by the previous GEMM together with per-row-tile
// partials {sum dy, sum (y - mean) dy}; dZ = (dy - S/M - (y - mean) D invstd^2 / M) invstd gamma.
#define CGL_BNB_TAB (CGL_BN_MAXF + 16)   // LDS table stride (floats; padding for the K-tail chunk)
struct CglBnBwdFold {
  const double* part;     // [tiles][F][2]
  int tiles, F, M;        // producer row tiles, features, rows of the BatchNorm call
  const float* mean; const float* invstd; const float* gamma;   // [F] (the call's saved statistics)
  float* g_gamma; float* g_beta;       // written by workgroup 0 of the k-contiguous problem
  const float* y; int ldy;             // BatchNorm input rows (same row / column positions as A)
};

struct CglGemmDesc {
  int M, N, K;
  int WM, WN, WK;         // wave arrangement, WM*WN*WK == 4
  int tiles_m, tiles_n;
  int wg_begin;           // first workgroup of this problem in a grouped launch
  int xcd_pm;             // XCD blocking: the tile grid is cut into xcd_pm x (8 / xcd_pm) slabs, slab x on XCD x
                          // (its L2 then holds 1 / xcd_pm of A and xcd_pm / 8 of B); 0 = n-major ranges
  int layout;             // 0: NT (A[m][k], B[n][k]); 1: NN (A[m][k], B[k][n]); 2: TN (A[k][m], B[k][n])
  int a_vec, b_vec;       // 16-byte vector loads allowed along each operand's contiguous dim
  int TM, TN;             // 32x32 accumulator blocks per wave (1x1 or 2x2)
  CglRowSrc a, b;
  int a_pk, b_pk;         // NT operand in the fragment-packed layout P (a.p0 / b.p0 = its base)
  // A copy-out (kc A only)
  float* a_copy;         // optional copy-out of the (transformed) A rows; rows >= a_copy_row0
  int a_copy_ld, a_copy_row0;
  // B extras
  int b_ones_col;         // logical column N-1 of B is all ones (bias-gradient trick)
  // epilogue
  float* C; int ldc;
  const float* bias;
  int act; float slope;
  const float* mask_ref; int mask_ld;     // v *= (ref > 0 ? 1 : slope)
  const float* tanh_ref; int tanh_ld;     // v *= 1 - t*t
  float* stat_part; int stat_gr;          // forward BatchNorm partials of the stored output
  float* bias_out;                     // with b_ones_col: column N-1 of C goes here
  // output row permutation (0: none): with lp = c_perm & 255, lq = c_perm >> 8, row r of the result is stored as
  // row ((r & (2^lp - 1)) << lq) + (r >> lp) of C (and of bias_out) -- the NHWC -> NCHW feature order of a weight
  // gradient whose A operand is an NHWC activation gradient (cgl_linear_prepare_wgrad_nhwc); plain stores only
  int c_perm;
  // cross-workgroup split-K (ksplit > 1): the K range is cut into ksplit slices, one workgroup per
  // (tile, slice); every slice stores its tile partial write-through (sc1) to kpart, the workgroup
  // that draws the last ticket of kcount[tile] sums the partials in slice order (deterministic),
  // runs the epilogue and re-zeroes the ticket
  int ksplit;
  float* kpart;                        // [ksplit][tiles][WM*WN][TM*TN][16][64] floats
  unsigned int* kcount;                // [tiles], zero at rest
  // A-operand transform (cgl_gemm.hip): 0 none, 1 forward BatchNorm1d + LeakyReLU (a_bnf),
  // 2 backward BatchNorm1d (a_bnb); its LDS tables take the first tab_floats of the dynamic LDS
  int a_bn;
  int tab_floats;
  CglBnFwd a_bnf;
  CglBnBwdFold a_bnb;
  // backward BatchNorm partials of the stored output dy: [tiles_m][N][2] {sum dy, sum (y - mean) dy}
  double* bnb_part;
  const float* bnb_y; int bnb_ld;      // the BatchNorm input at the stored positions
  const float* bnb_mean;               // its saved batch mean [N]
  // dynamic loss scaling (16-bit instantiations only): a stored non-finite value raises *inf_flag
  unsigned int* inf_flag;
  // epilogue Adam (the ADAM instantiation: G's first-layer weight gradient fused with the G Adam launch):
  // the parameter / moment tensors parallel to C (ad_p ...) and to bias_out (ad_pb ...), updated with
  // cgl_adam_update from the stored gradient value, as cgl_adam would from memory
  // A generated in the prologue of the launch (a_gen: the round prologue fused with G's first GEMM): the
  // workgroup first draws the N(0,1) rows of its tile into a.p0 (cgl_normal_at, round *gen_round + 1,
  // stream 0, gen_n floats in all) -- the z the separate prologue launch drew
  int a_gen;
  const int* gen_round;
  unsigned long long gen_seed;
  long gen_n;
  float* ad_p; float* ad_m; float* ad_v;
  float* ad_pb; float* ad_mb; float* ad_vb;
  const float* ad_ss; const float* ad_bc;
  float ad_b2, ad_w1, ad_w2, ad_eps;
  const struct CglHeadDesc* fin_head;   // desc 0 of a launch: the previous head launch's deferred loss reduction,
                                         // run by one extra workgroup (the launch's last)
  // diagnostics (builds with -DCGL_GEMM_TRACE only, env CGL_GEMM_TRACE=1): per workgroup of this problem,
  // CGL_GEMM_TRACE_W wall-clock stamps (100 MHz, tools/gemm_trace.py)
  unsigned long long* trace;
};
// Problem selection of a grouped GEMM launch (cgl_gemm_f32 kernel arguments; at most 3 problems per launch)
struct CglGemmSel {
  int wg1, wg2;     // first workgroup of problems 1 and 2 (INT_MAX: absent)
  int meta;         // per problem q: (layout | (a_vec && b_vec) << 2) << 4 q
  int fin;          // problem 0 carries fin_head (the previous head launch's deferred loss reduction)
  // (host side only) the next GEMM launch's descriptors, from 128-byte line pf, pf_lines lines: warmed into
  // every XCD's L2 by this launch (cgl_gemm_f32's pf / pf_lines arguments; nullptr / 0: none)
  const int* pf = nullptr;
  int pf_lines = 0;
};
#define CGL_GEMM_TRACE_WGS 4096   // workgroups per problem with trace slots
#ifdef CGL_GEMM_TRACE_CHUNKS      // + wave 0's stamp after each of its first 64 chunks (words 8 ..)
#define CGL_GEMM_TRACE_W 72
#else
#define CGL_GEMM_TRACE_W 8        // words per workgroup: kernel entry, body, k-loop start, chunk 0 consumed,
#endif                            // k-loop end, exit

// BatchNorm1d(train) + LeakyReLU over the whole [mtot][F] output of one G layer.
struct CglBnApplyDesc {
  int F;
  const float* Y; int ld_y;       // pre-BN (Linear output)
  float* act; int ld_act;         // post-LeakyReLU
  float* act_pk;                  // the same in the fragment-packed layout P(act; mtot, F), or null
  CglBnFwd bn;
};

// D output layer + adversarial loss (+ its backward into the last hidden layer).
struct CglHeadDesc {
  int M, F, C;            // rows, input features, logits (2: CE, 1: Sigmoid+BCE)
  int loss;               // 0 CE, 1 BCE
  const float* P; int ldp;        // last hidden activations (post-LeakyReLU) [M][F]
  const float* W; const float* b; // [C][F], [C]
  int split;              // rows < split: target t0 weight w0; others: t1, w1
  int t0, t1;
  float w0, w1;           // dlogit scale per segment (mean and the 0.5 of D_loss folded in)
  float* dlogits;         // [M][C] (optional)
  float* dP; int lddp;    // (dlogits . W) * leaky'(P)
  float slope;
  const int* n0_dev;      // when set: segment 0 has only *n0_dev valid rows (the rest carry no loss and
                          // no gradient) and its mean / dlogit weight use that count (w0 = combine / n0)
  float* part;            // [nwg][2] per-workgroup loss sums per segment
  unsigned int* counter;  // last-arriver ticket (zero at rest)
  float* loss_out0;       // mean loss of segment 0 / 1 (written by the last workgroup), may be null
  float* loss_out1;
  float* loss_out2;       // a second copy of segment 0's mean (the exchange slot's loss word), may be null
  const float* scale_dev; // dynamic loss scaling: the dlogits (and dP) carry this factor, the loss does not
  float combine;          // D_loss = (seg0 + seg1) * combine  (0.5: capgan.py:339, 1: CGLGAN/2DMG/main.py:364)
  float* combine_out;     // optional
  const float* combine_in0;  // segment-0 mean computed by another launch (when this one has no segment 0)
  int rows_per_wg;
  int deferred;           // the batch-mean reduction is left to the next GEMM launch's finisher workgroup
  int nwg;                // (deferred) this launch's workgroups = partials to reduce
};
// batch-mean loss reduction of a head launch's partials (cgl_kernels.hip; also run by a GEMM finisher workgroup)
__device__ void cgl_head_finish(const CglHeadDesc* __restrict__ hd, int nwg, float* s_part);


// Standalone BatchNorm1d forward (nn.Module path): batch or running statistics, optional LeakyReLU.
struct CglBn1dDesc {
  int M, F, ldx, train, act;
  const float* X; float* Y;
  const float* gamma; const float* beta;
  double eps, momentum;
  float slope;
  float* run_mean; float* run_var; float* save_mean; float* save_invstd;
};

// BatchNorm1d backward for one layer, fused with the LeakyReLU mask of its output (post may be
// null: no activation).
struct CglBnBwdDesc {
  int M, F;
  const float* dA; int ld_da;     // gradient w.r.t. the LeakyReLU output
  const float* post; int ld_post; // LeakyReLU output (mask source)
  const float* Y; int ld_y;       // BatchNorm input (pre-BN)
  const float* mean; const float* invstd; const float* gamma;
  float* dZ; int ld_dz;           // gradient w.r.t. the BatchNorm input
  float* dZ_pk;                   // the same in the fragment-packed layout P(dZ; M, F), or null
  float* g_gamma; float* g_beta;
  float slope;
  // dynamic loss scaling: a non-finite dgamma / dbeta raises *inf_flag (the model's found word, as the
  // 16-bit GEMM weight-gradient epilogues do for W / b), so GradScaler's check covers every gradient
  unsigned int* inf_flag;
};

#define CGL_MAX_EPOCH 8
#define CGL_MAX_WORKERS 64

// Per-context device scalar block.  Written only by cgl_step_begin (counters, Adam bias
// corrections), by the head kernels' last workgroup (losses), by cgl_alpha_scale and by
// the scalar tail of the G Adam launch; every other kernel only reads it.
struct CglStepState {
  int round;                        // rounds started
  int n_workers, rank, weighting;   // exchange configuration
  float g_step_size, g_bc2sqrt;     // Adam bias corrections for this round's G update
  float d_step_size[CGL_MAX_EPOCH], d_bc2sqrt[CGL_MAX_EPOCH];
  float lambda;                     // CAPGAN / Mix-G / CGLGAN lambda
  float d_loss_parts[CGL_MAX_EPOCH][2];  // mean real / fake loss of each local D step
  float d_loss[CGL_MAX_EPOCH];
  float g_loss_parts[2];            // [0] = own G loss (mean over rows)
  float alpha;                      // weight applied to the own G-loss gradient
  float F;                          // F_max reported by the reference's Server.train
  float beta[CGL_MAX_WORKERS];      // data-size weights
  float losses[CGL_MAX_WORKERS];    // gathered G losses (N > 1)
  float alphas[CGL_MAX_WORKERS];
  long long bn_batches;             // num_batches_tracked of every G BatchNorm layer
  int real_rows[CGL_MAX_EPOCH];     // real rows of each local D step's batch (device sampler: the
                                    // pass's short last batch has fewer, capgan.py:326-331)
  // dynamic loss scaling (cgl_gan_config.loss_scale > 0), index 0 = D, 1 = G.  The round's GEMM
  // epilogues raise found[m] when they store a non-finite weight gradient, the Adam launch of model m
  // skips its step when found[m] is set; the NEXT round's prologue applies GradScaler.update (scale,
  // growth tracker, torch's Adam step count adam_t) and clears found (scaler_pending, set by the G-Adam
  // tail, marks that a round has ended since)
  float scale[2];
  unsigned int found[2];
  int growth[2];
  int adam_t[2];
  int skipped[2];
  int last_skipped[2];
  int scaler_pending;
  unsigned int err;                 // sticky: an in-launch rendezvous timed out (never expected)
  int cur_round;                    // the round in progress (1-based; written by its prologue): the G Adam
                                    // launch draws the NEXT round's z with counter cur_round + 1
};

enum { CGL_W_CAPGAN = 0, CGL_W_MEAN = 1, CGL_W_MIX_SINGLE = 2, CGL_W_MIX_DOUBLE = 3, CGL_W_CGLGAN = 4 };

#include "cgl_common.h"
