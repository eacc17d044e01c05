// Host runtime of libcglgan_hip: plans one CGL-GAN communication round as a fixed list of
// kernel launches over caller-owned buffers, and replays it eagerly or through a hipGraph.
//
// Replaces the reference's Python role loop: Server.train (capgan.py:211-262,
// mixed-gan.py:238-292, MDGAN/MNIST/mdgan.py:180-207, CGLGAN/2DMG/main.py:225-278) and
// Worker.train (capgan.py:316-349, mixed-gan.py:355-392, MDGAN/MNIST/mdgan.py:266-297,
// CGLGAN/2DMG/main.py:344-375) -- on ONE device per worker, with G replicated per worker and
// the reference's queue exchange turned into an all-reduce between phase A and phase B.
//
// The non-GEMM kernels are compiled in this translation unit, the GEMM kernel instances in cgl_gemm_inst.hip.
#include "cgl_gemm.hip"
#include "cgl_kernels.hip"
#include "cgl_round.h"
#include "../../include/cglgan.h"

// the GEMM kernels are instantiated in the cgl_gemm_inst.hip translation units (compiled in parallel):
// declared here so that this unit only launches them
#define CGL_INST_PREFIX extern template
#include "cgl_gemm_inst.h"

#include <hip/hip_ext.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#define CGL_VERSION_STR "0.1.0 gfx950"

namespace {

inline int64_t al64(int64_t n) { return (n + 63) & ~int64_t(63); }

struct TensorRec {
  int64_t off;
  int rows, cols, layer, kind;  // kind: 0 W, 1 b, 2 BN gamma, 3 BN beta
};

std::vector<TensorRec> param_layout(const cgl_mlp_spec& s, int64_t* total) {
  std::vector<TensorRec> v;
  int64_t off = 0;
  for (int l = 0; l < s.n_layers; ++l) {
    const int fo = s.dims[l + 1], fi = s.dims[l];
    v.push_back({off, fo, fi, l, 0});
    off += al64((int64_t)fo * fi);
    v.push_back({off, fo, 1, l, 1});
    off += al64(fo);
    if (s.bn[l]) {
      v.push_back({off, fo, 1, l, 2});
      off += al64(fo);
      v.push_back({off, fo, 1, l, 3});
      off += al64(fo);
    }
  }
  if (total) *total = off;
  return v;
}

int64_t running_layout(const cgl_mlp_spec& s, int64_t* mean_off, int64_t* var_off) {
  int64_t off = 0;
  for (int l = 0; l < s.n_layers; ++l) {
    if (mean_off) mean_off[l] = -1;
    if (var_off) var_off[l] = -1;
    if (!s.bn[l]) continue;
    if (mean_off) mean_off[l] = off;
    off += al64(s.dims[l + 1]);
    if (var_off) var_off[l] = off;
    off += al64(s.dims[l + 1]);
  }
  return off;
}

constexpr int kHeadRows = 4;     // one row per wave of a head workgroup

int validate(const cgl_gan_config* c) {
  if (!c) return CGL_E_ARG;
  const cgl_mlp_spec &g = c->g, &d = c->d;
  if (g.n_layers < 1 || g.n_layers > CGL_MAX_LAYERS || d.n_layers < 2 || d.n_layers > CGL_MAX_LAYERS)
    return CGL_E_ARG;
  for (int l = 0; l <= g.n_layers; ++l)
    if (g.dims[l] < 1) return CGL_E_ARG;
  for (int l = 0; l <= d.n_layers; ++l)
    if (d.dims[l] < 1) return CGL_E_ARG;
  if (g.dims[g.n_layers] != d.dims[0]) return CGL_E_ARG;
  if (g.bn[g.n_layers - 1]) return CGL_E_ARG;
  for (int l = 0; l < d.n_layers; ++l)
    if (d.bn[l]) return CGL_E_ARG;
  const int C = d.dims[d.n_layers];
  if (c->loss == CGL_LOSS_CE2 && C != 2) return CGL_E_ARG;
  if (c->loss == CGL_LOSS_BCE && C != 1) return CGL_E_ARG;
  if (d.dims[d.n_layers - 1] % 4 != 0) return CGL_E_ARG;  // loss head reads 16-byte vectors
  if (d.dims[d.n_layers - 1] > 4 * 64 * CGL_HEAD_MAXQ) return CGL_E_ARG;  // head keeps a row in registers
  if ((c->batch_real + c->batch + kHeadRows - 1) / kHeadRows > 1024) return CGL_E_ARG;  // head partials in LDS
  if (c->loss != CGL_LOSS_CE2 && c->loss != CGL_LOSS_BCE) return CGL_E_ARG;
  if (c->batch < 2 || c->batch_real < 1 || c->epoch < 1 || c->epoch > CGL_MAX_EPOCH) return CGL_E_ARG;
  if (c->n_workers < 1 || c->n_workers > CGL_MAX_WORKERS || c->rank < 0 || c->rank >= c->n_workers)
    return CGL_E_ARG;
  if (c->weighting < 0 || c->weighting > 4) return CGL_E_ARG;
  if (c->exchange_layer != -1 && (c->exchange_layer < 1 || c->exchange_layer >= g.n_layers)) return CGL_E_ARG;
  if (c->sample_n < 0) return CGL_E_ARG;
  if (c->gemm_dtype < CGL_DTYPE_F32 || c->gemm_dtype > CGL_DTYPE_BF16) return CGL_E_ARG;
  // dynamic loss scaling: 16-bit GEMM operands only, one local D step per round, S a power of two (the
  // unscale 1 / S is then exact), a non-negative growth interval
  if (c->loss_scale < 0.f || c->scale_growth_interval < 0) return CGL_E_ARG;
  if (c->loss_scale > 0.f) {
    int ex = 0;
    if (!std::isfinite(c->loss_scale) || std::frexp(c->loss_scale, &ex) != 0.5f) return CGL_E_ARG;
    if (c->gemm_dtype == CGL_DTYPE_F32 || c->epoch != 1) return CGL_E_ARG;
  }
  return CGL_OK;
}

// ----------------------------------------------------------------------------------------
// workspace carve (sizing pass with base == nullptr)
struct Carve {
  char* base;
  int64_t off = 0;
  explicit Carve(void* b) : base((char*)b) {}
  template <class T>
  T* take(int64_t count) {
    const int64_t bytes = (count * (int64_t)sizeof(T) + 255) & ~int64_t(255);
    T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
    off += bytes;
    return p;
  }
};

constexpr int kMaxGemmDescs = 128;
constexpr int64_t kTraceWords = CGL_GEMM_TRACE_W * CGL_GEMM_TRACE_WGS;   // CGL_GEMM_TRACE stamps
constexpr int kMaxHeadDescs = 2 * CGL_MAX_EPOCH + 4;
constexpr int kMaxBnDescs = 2 * CGL_MAX_LAYERS;
constexpr int kSplitKCounters = 8192;           // split-K tickets (one per tile of a launch)
constexpr int kCounters = 64;                    // head-loss tickets
constexpr int64_t kSplitKFloats = 4 << 20;       // split-K partials of one launch (16 MiB)

// An exchange buffer (dYL, or a Mix-G trunk gradient gdA / gG) is followed by kXchgPad floats: the gathered
// exchange (cgl_gan_exchange_mode 1) sends [gradient | G loss | padding] as one slot of xchg_slot(n) floats.
constexpr int64_t kXchgPad = 64;
inline int64_t xchg_slot(int64_t n) { return (n + 1 + 63) & ~(int64_t)63; }
inline int64_t xchg_slot_max(const cgl_gan_config& c) {
  int f = c.g.dims[c.g.n_layers];
  for (int l = 1; l < c.g.n_layers; ++l) f = std::max(f, c.g.dims[l]);
  return xchg_slot((int64_t)c.batch * f);
}

struct WS {
  float* znext;                     // z_ahead: the next round's z [2B][z_dim], drawn by the G Adam launch
  // G forward (2B rows)
  float* gout[CGL_MAX_LAYERS];
  float* gact[CGL_MAX_LAYERS];
  float* gpart[CGL_MAX_LAYERS];
  float* gmean[CGL_MAX_LAYERS];
  float* ginvstd[CGL_MAX_LAYERS];
  // D step (Md rows)
  float* R;
  float* P[CGL_MAX_LAYERS];
  float* dQ[CGL_MAX_LAYERS];
  float* dlog;
  // D(Xg) (B rows)
  float* S[CGL_MAX_LAYERS];
  float* dS[CGL_MAX_LAYERS];
  float* dYL;
  // G backward (B rows)
  float* gdA[CGL_MAX_LAYERS];
  float* gG[CGL_MAX_LAYERS];
  // misc
  float* hpart;
  float* hpart2;
  unsigned int* counters;   // [kCounters]: head-loss tickets
  float* kpart;             // [kSplitKFloats]: split-K partials (reused by every launch)
  unsigned int* kcount;     // [kSplitKCounters]: split-K tickets (zero at rest)
  double* gdpart[CGL_MAX_LAYERS];   // backward BatchNorm partials of dy [B/32][f][2] (a_bn 2)
  float* gpk[CGL_MAX_LAYERS];       // packed BatchNorm + LeakyReLU output P(act_l; 2B, f) (next GEMM's A)
  float* wpk[CGL_MAX_LAYERS];       // packed G weights P(W_l; fo, fi) (the forward GEMM's B)
  float* wtpk[CGL_MAX_LAYERS];      // packed transposed G weights P(W_l^T; fi, fo) (input-gradient B)
  float* gGpk[CGL_MAX_LAYERS];      // packed cgl_bn_bwd output P(dZ_l; B, f) (input-gradient A)
  float* dwpk[CGL_MAX_LAYERS];      // packed D weights P(V_j; fo, fi) (the D forward GEMMs' B), written by D's Adam
  float* dwtpk[CGL_MAX_LAYERS];     // packed transposed D weights P(V_j^T; fi, fo) (the D input gradients' B)
  float* gath;                      // gathered exchange: n_workers slots of xchg_slot_max() floats
  CglStepState* st;
  int* idx;       // sampler output when sample_n > 0
  CglGemmDesc* gemm;
  CglHeadDesc* head;
  CglBnBwdDesc* bnb;
  CglBnApplyDesc* bna;
  int64_t total;
};

WS carve_ws(const cgl_gan_config& c, void* base) {
  WS w;
  std::memset(&w, 0, sizeof(w));
  Carve cv(base);
  const cgl_mlp_spec &g = c.g, &d = c.d;
  const int L = g.n_layers, J = d.n_layers;
  const int B = c.batch, Md = c.batch_real + c.batch;
  w.st = cv.take<CglStepState>(1);
  w.counters = cv.take<unsigned int>(kCounters);
  w.gemm = cv.take<CglGemmDesc>(kMaxGemmDescs);
  w.head = cv.take<CglHeadDesc>(kMaxHeadDescs);
  w.bnb = cv.take<CglBnBwdDesc>(kMaxBnDescs);
  w.bna = cv.take<CglBnApplyDesc>(kMaxBnDescs);
  for (int l = 0; l < L; ++l) {
    const int f = g.dims[l + 1];
    w.gout[l] = cv.take<float>((int64_t)2 * B * f);
    if (l + 1 < L && g.bn[l]) {
      w.gact[l] = cv.take<float>((int64_t)2 * B * f);
      const int64_t tiles = (2 * B + 31) / 32;
      w.gpart[l] = cv.take<float>(tiles * 2 * f * 2);
      w.gmean[l] = cv.take<float>((int64_t)2 * f);
      w.ginvstd[l] = cv.take<float>((int64_t)2 * f);
      w.gdA[l] = cv.take<float>((int64_t)B * f + kXchgPad);
    }
    if (l + 1 < L) w.gG[l] = cv.take<float>((int64_t)B * f + kXchgPad);
  }
  w.R = cv.take<float>((int64_t)Md * d.dims[0]);
  for (int j = 0; j + 1 < J; ++j) {
    const int f = d.dims[j + 1];
    w.P[j] = cv.take<float>((int64_t)Md * f);
    w.dQ[j] = cv.take<float>((int64_t)Md * f);
    w.S[j] = cv.take<float>((int64_t)B * f);
    w.dS[j] = cv.take<float>((int64_t)B * f);
  }
  w.dlog = cv.take<float>((int64_t)Md * d.dims[J]);
  w.dYL = cv.take<float>((int64_t)B * g.dims[L] + kXchgPad);
  w.hpart = cv.take<float>((int64_t)((Md + kHeadRows - 1) / kHeadRows) * 2);
  w.hpart2 = cv.take<float>((int64_t)((Md + kHeadRows - 1) / kHeadRows) * 2);
  w.idx = cv.take<int>((int64_t)c.epoch * c.batch_real);
  w.znext = cv.take<float>((int64_t)2 * B * g.dims[0]);
  w.gath = cv.take<float>((int64_t)std::max(c.n_workers, 1) * xchg_slot_max(c));
  for (int j = 0; j + 1 < J; ++j) {
    w.dwpk[j] = cv.take<float>(cgl_pk_floats(d.dims[j + 1], d.dims[j]));
    w.dwtpk[j] = cv.take<float>(cgl_pk_floats(d.dims[j], d.dims[j + 1]));
  }
  // split-K scratch last, so that the layout of everything the default plan touches is unchanged
  w.kpart = cv.take<float>(kSplitKFloats);
  w.kcount = cv.take<unsigned int>(kSplitKCounters);
  for (int l = 0; l + 1 < L; ++l)
    if (g.bn[l]) w.gdpart[l] = cv.take<double>((int64_t)((B + 31) / 32) * g.dims[l + 1] * 2);
  for (int l = 0; l < L; ++l) {
    if (l + 1 < L && g.bn[l]) w.gpk[l] = cv.take<float>(cgl_pk_floats(2 * B, g.dims[l + 1]));
    w.wpk[l] = cv.take<float>(cgl_pk_floats(g.dims[l + 1], g.dims[l]));
    if (l >= 1) w.wtpk[l] = cv.take<float>(cgl_pk_floats(g.dims[l], g.dims[l + 1]));
    if (l + 1 < L && g.bn[l]) w.gGpk[l] = cv.take<float>(cgl_pk_floats(B, g.dims[l + 1]));
  }
  w.total = cv.off;
  return w;
}

// ----------------------------------------------------------------------------------------
enum LaunchKind { K_GEMM, K_HEAD, K_BNBWD, K_ADAM, K_PROLOGUE, K_BNAPPLY, K_GEMM_ADAM, K_GEMM_PRO, K_COMBINE };

struct Launch {
  LaunchKind kind;
  int grid = 1;
  int grid_y = 1;
  int first = 0, count = 0;  // descriptor range (host index)
  CglAdamArgs adam{};
  int tail = 0;
  CglBeginArgs begin{};
  float* nptr = nullptr;  // prologue: z buffer, its length, normal / sampler block counts
  long nn = 0;
  int nb_norm = 0, nb_samp = 0;
  int stream_id = 0;
  double flops = 0.0;
  int stream = 0;       // 0: the caller's stream, 1: the context's side stream
  int wait_ev = -1;     // event waited on before the launch / recorded after it
  int record_ev = -1;
  int shmem = 0;        // dynamic LDS bytes (GEMM)
  int blk = 1;          // GEMM per-wave block shape (TM = TN = blk)
  bool sk = false;      // GEMM launch holds a split-K problem
  int dt = CGL_DTYPE_F32;   // GEMM operand type (cgl_gan_config.gemm_dtype)
  int abn = 0;              // GEMM operand-transform instantiation (the launch's a_bn)
  bool adpk = false;        // K_ADAM: the cgl_adam_pack form (cgl_gan.adam_pack, or adam_pack_d for D's Adam)
  int apk_d = 0;            // K_ADAM adpk: 1 = D's (cgl_gan.adam_pack_d)
  bool v4 = false;          // K_ADAM (not adpk): the four-elements-per-thread form (cgl_adam4)
  int layer = -1;           // K_BNAPPLY: the G layer whose forward GEMM reads this launch's output
  int pk = -1;              // K_BNAPPLY: index of the packing jobs it carries (cgl_gan.carry), -1: none
  int pf_first = -1, pf_count = 0;   // K_GEMM: the next GEMM launch's descriptor range (link_gemm_prefetch)
};

// Every kernel of a plan is launched through klaunch.  Normally a plain launch; while cgl_gan_profile
// runs a round, each launch carries a start / stop event pair (hipExtLaunchKernelGGL): the events take
// the dispatch's own begin / end timestamps -- the interval rocprofv3's kernel trace reports -- so the
// per-launch durations of a round need no extra barrier packets between the launches.
thread_local hipEvent_t t_prof_ev[2] = {nullptr, nullptr};

template <typename... KArgs, typename... Args>
void klaunch(void (*k)(KArgs...), dim3 grid, dim3 block, uint32_t shmem, hipStream_t s, Args... args) {
  if (t_prof_ev[0])
    hipExtLaunchKernelGGL(k, grid, block, shmem, s, t_prof_ev[0], t_prof_ev[1], 0u, ((KArgs)args)...);
  else
    hipLaunchKernelGGL(k, grid, block, shmem, s, ((KArgs)args)...);
}

// Split-K partials of 2x2-block waves need up to 48 KB of dynamic LDS (+ the 20 KB operand tables).
hipError_t gemm_lds_attr() {
  static bool done = false;
  if (!done) {
    // advisory on this platform (launches up to the per-CU LDS succeed); never fail on it
    for (const void* fn : {(const void*)cgl_gemm_f32<1, 1>, (const void*)cgl_gemm_f32<2, 2>,
                           (const void*)cgl_gemm_f32<1, 1, true>, (const void*)cgl_gemm_f32<2, 2, true>,
                           (const void*)cgl_gemm_f32<1, 1, false, CGL_DTYPE_F32, 1>,
                           (const void*)cgl_gemm_f32<2, 2, false, CGL_DTYPE_F32, 1>,
                           (const void*)cgl_gemm_f32<1, 1, false, CGL_DTYPE_F32, 2>,
                           (const void*)cgl_gemm_f32<2, 2, false, CGL_DTYPE_F32, 2>}) {
      for (int kb : {150, 128, 96, 64}) {
        const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, kb * 1024);
        (void)hipGetLastError();
        if (e == hipSuccess) break;
      }
    }
    done = true;
  }
  return hipSuccess;
}

template <int DT>
void launch_gemm16(int blk, int grid, int shmem, hipStream_t s, const CglGemmDesc* d, CglGemmSel n, bool sk) {
  if (sk) {
    if (blk == 2)
      klaunch(cgl_gemm_f32<2, 2, true, DT>, dim3(grid), dim3(CGL_GEMM_THREADS), shmem, s, d, n.wg1, n.wg2, n.meta, n.fin, n.pf, n.pf_lines);
    else
      klaunch(cgl_gemm_f32<1, 1, true, DT>, dim3(grid), dim3(CGL_GEMM_THREADS), shmem, s, d, n.wg1, n.wg2, n.meta, n.fin, n.pf, n.pf_lines);
  } else if (blk == 2) {
    klaunch(cgl_gemm_f32<2, 2, false, DT>, dim3(grid), dim3(CGL_GEMM_THREADS), shmem, s, d, n.wg1, n.wg2, n.meta, n.fin, n.pf, n.pf_lines);
  } else {
    klaunch(cgl_gemm_f32<1, 1, false, DT>, dim3(grid), dim3(CGL_GEMM_THREADS), shmem, s, d, n.wg1, n.wg2, n.meta, n.fin, n.pf, n.pf_lines);
  }
}

// The problem selection of a launch (CglGemmSel) from the host copies of its n problems.
CglGemmSel gemm_sel(const CglGemmDesc* hd, int n) {
  CglGemmSel q;
  q.wg1 = n > 1 ? hd[1].wg_begin : INT_MAX;
  q.wg2 = n > 2 ? hd[2].wg_begin : INT_MAX;
  q.meta = 0;
  for (int i = 0; i < n && i < 3; ++i) q.meta |= (hd[i].layout | ((hd[i].a_vec && hd[i].b_vec) ? 4 : 0)) << (4 * i);
  q.fin = hd[0].fin_head ? 1 : 0;
  return q;
}

// d: the device descriptors of the launch, n: their selection (gemm_sel of the host copies)
void launch_gemm(int blk, int grid, int shmem, hipStream_t s, const CglGemmDesc* d, CglGemmSel n, bool sk = false,
                 int dt = CGL_DTYPE_F32, int abn = 0) {
  if (abn == 1) {          // fp32, no split-K (planner)
    if (blk == 2)
      klaunch(cgl_gemm_f32<2, 2, false, CGL_DTYPE_F32, 1>, dim3(grid), dim3(CGL_GEMM_THREADS), shmem, s, d, n.wg1, n.wg2, n.meta, n.fin, n.pf, n.pf_lines);
    else
      klaunch(cgl_gemm_f32<1, 1, false, CGL_DTYPE_F32, 1>, dim3(grid), dim3(CGL_GEMM_THREADS), shmem, s, d, n.wg1, n.wg2, n.meta, n.fin, n.pf, n.pf_lines);
  } else if (abn == 2) {
    if (blk == 2)
      klaunch(cgl_gemm_f32<2, 2, false, CGL_DTYPE_F32, 2>, dim3(grid), dim3(CGL_GEMM_THREADS), shmem, s, d, n.wg1, n.wg2, n.meta, n.fin, n.pf, n.pf_lines);
    else
      klaunch(cgl_gemm_f32<1, 1, false, CGL_DTYPE_F32, 2>, dim3(grid), dim3(CGL_GEMM_THREADS), shmem, s, d, n.wg1, n.wg2, n.meta, n.fin, n.pf, n.pf_lines);
  } else if (dt == CGL_DTYPE_F16) {
    launch_gemm16<CGL_DTYPE_F16>(blk, grid, shmem, s, d, n, sk);
  } else if (dt == CGL_DTYPE_BF16) {
    launch_gemm16<CGL_DTYPE_BF16>(blk, grid, shmem, s, d, n, sk);
  } else if (sk) {   // a launch with a split-K problem: the instantiation carrying the combine
    if (blk == 2)
      klaunch(cgl_gemm_f32<2, 2, true>, dim3(grid), dim3(CGL_GEMM_THREADS), shmem, s, d, n.wg1, n.wg2, n.meta, n.fin, n.pf, n.pf_lines);
    else
      klaunch(cgl_gemm_f32<1, 1, true>, dim3(grid), dim3(CGL_GEMM_THREADS), shmem, s, d, n.wg1, n.wg2, n.meta, n.fin, n.pf, n.pf_lines);
  } else if (blk == 2) {
    klaunch(cgl_gemm_f32<2, 2>, dim3(grid), dim3(CGL_GEMM_THREADS), shmem, s, d, n.wg1, n.wg2, n.meta, n.fin, n.pf, n.pf_lines);
  } else {
    klaunch(cgl_gemm_f32<1, 1>, dim3(grid), dim3(CGL_GEMM_THREADS), shmem, s, d, n.wg1, n.wg2, n.meta, n.fin, n.pf, n.pf_lines);
  }
}

// Cost model of one GEMM launch (cycles) used to pick the wave arrangement WM x WN x WK and
// the per-wave block shape TM x TN:
//   MFMA issue per SIMD, one wave's dependent chain incl. the part of the memory latency its
//   (S-1)-deep prefetch does not cover, and the per-CU address/L1 rate of the fragment loads
//   (a fragment load touches 32 cache lines), plus the split-K reduction.
//   KS > 1: cross-workgroup split-K -- KS times the workgroups, 1 / KS of the chunks each, plus
//   the combine (publish, ticket, the reducer's read of KS partials).
double gemm_cost(int M, int N, int K, int WM, int WN, int WK, int TM, int TN, int KS = 1, double ta_a = 1.0,
                 double ta_b = 1.0) {
  const double lat = 2000.0;
  const int S = 3;
  const long tiles = (long)((M + 32 * TM * WM - 1) / (32 * TM * WM)) * ((N + 32 * TN * WN - 1) / (32 * TN * WN));
  const double wg_per_cu = std::ceil(tiles * KS / 256.0);
  const int nch = (K + CGL_GEMM_KCHUNK - 1) / CGL_GEMM_KCHUNK;
  const double per = std::ceil((double)nch / (WK * KS));
  const double blk = 512.0 * TM * TN;
  const double mfma = wg_per_cu * per * blk;
  const double chain = per * std::max(blk, lat / (S - 1));
  // a fragment load of a row-major k-contiguous operand touches 32 lines, a packed one 8 (ta_x = 1 / 0.25)
  const double ta = wg_per_cu * 4 * per * (TM * ta_a + TN * ta_b) * 64.0;
  return std::max(mfma, std::max(chain, ta)) + (WK > 1 ? 400.0 * TM * TN : 0.0) +
         (KS > 1 ? 2400.0 + 300.0 * KS * TM * TN : 0.0);
}

// Cross-workgroup split-K factor for a chosen tile shape (CGL_SPLITK=0 disables, =N forces N):
// KS in {1, 2, 4} with >= 2 chunks per wave and a partial slab of <= 16 KB per tile.
int gemm_splitk_env() {
  static int v = -2;
  if (v == -2) {
    const char* e = getenv("CGL_SPLITK");
    v = e ? atoi(e) : 0;
  }
  return v;
}
void choose_ks(CglGemmDesc& d) {
  d.ksplit = 1;
  // Measured on MI355X (tools/gemm_bench REPS 2, profiles/r01_gemm_microbench_v8_splitk.txt): the
  // combine (publish + ticket + the reducer's read, ~2-3 us) outweighs the shorter k-loop on every
  // GEMM of the B=256 round, so split-K is opt-in (CGL_SPLITK=N forces N; -1 = cost model).
  const int env = gemm_splitk_env();
  if (env == 0) return;
  const int nch = (d.K + CGL_GEMM_KCHUNK - 1) / CGL_GEMM_KCHUNK;
  const long slab = (long)d.WM * d.WN * d.TM * d.TN * 4096;
  if (slab > 16384) return;
  double best = gemm_cost(d.M, d.N, d.K, d.WM, d.WN, d.WK, d.TM, d.TN, 1);
  for (int ks : {2, 4}) {
    if (nch < 2 * d.WK * ks) break;
    if (env > 0 && ks != env) continue;
    const double c = gemm_cost(d.M, d.N, d.K, d.WM, d.WN, d.WK, d.TM, d.TN, ks);
    if (env > 0 || c < best * 0.97) {
      best = c;
      d.ksplit = ks;
    }
  }
}

// force_wm: rows per wave-row group fixed (32 * TM * WM == 32 * force_wm); force_t: TM = TN fixed
// CGL_GEMM_TILE="WM,WN,WK,T" forces one wave arrangement and block shape on every problem the
// planner tiles freely (tile-search experiments, profiles/r02_gemm_tile_search*.txt; unset = the
// cost model)
bool gemm_tile_env(int* o) {
  static int v[5] = {-1, 0, 0, 0, 0};
  if (v[0] < 0) {
    v[0] = 0;
    const char* e = getenv("CGL_GEMM_TILE");
    if (e && sscanf(e, "%d,%d,%d,%d", &v[1], &v[2], &v[3], &v[4]) == 4 && v[1] * v[2] * v[3] == 4 &&
        (v[4] == 1 || v[4] == 2))
      v[0] = 1;
  }
  for (int i = 0; i < 4; ++i) o[i] = v[i + 1];
  return v[0] == 1;
}

void choose_tiles(CglGemmDesc& d, int force_wm = 0, int force_t = 0) {
  static const int opts[4][3] = {{2, 2, 1}, {2, 1, 2}, {1, 2, 2}, {1, 1, 4}};
  double best = 1e300;
  int fe[4];
  if (!force_wm && !force_t && gemm_tile_env(fe)) {
    d.WM = fe[0];
    d.WN = fe[1];
    d.WK = fe[2];
    d.TM = d.TN = fe[3];
    d.tiles_m = (d.M + 32 * fe[3] * fe[0] - 1) / (32 * fe[3] * fe[0]);
    d.tiles_n = (d.N + 32 * fe[3] * fe[1] - 1) / (32 * fe[3] * fe[1]);
    return;
  }
  for (int t = 1; t <= 2; ++t) {
    if (force_t && t != force_t) continue;
    for (auto& o : opts) {
      if (force_wm && o[0] * t != force_wm) continue;
      const double c = gemm_cost(d.M, d.N, d.K, o[0], o[1], o[2], t, t, 1, d.a_pk ? 0.25 : 1.0, d.b_pk ? 0.25 : 1.0);
      if (c < best * (1.0 - 1e-9)) {
        best = c;
        d.WM = o[0];
        d.WN = o[1];
        d.WK = o[2];
        d.TM = d.TN = t;
        d.tiles_m = (d.M + 32 * t * o[0] - 1) / (32 * t * o[0]);
        d.tiles_n = (d.N + 32 * t * o[1] - 1) / (32 * t * o[1]);
      }
    }
  }
}

CglGemmDesc make_gemm(int layout, int M, int N, int K) {
  CglGemmDesc d;
  std::memset(&d, 0, sizeof(d));
  d.layout = layout;
  d.M = M;
  d.N = N;
  d.K = K;
  d.a.split = 0x7fffffff;
  d.b.split = 0x7fffffff;
  d.slope = 0.2f;
  d.act = CGL_EPI_ACT_NONE;
  choose_tiles(d);
  return d;
}

inline bool al16p(const void* p) { return ((uintptr_t)p & 15) == 0; }

// 16-byte loads are legal for an operand when every row start is 16-byte aligned and the
// contiguous extent is a multiple of 4 floats (k for k-contiguous operands, columns otherwise).
void set_vec(CglGemmDesc& d) {
  auto src_ok = [](const CglRowSrc& r) {
    return (r.ld % 4 == 0) && al16p(r.p0) && (r.p1 == nullptr || al16p(r.p1));
  };
  const int nmem = d.N - (d.layout != 0 ? d.b_ones_col : 0);
  if (d.layout == 0) {
    d.a_vec = d.a_pk || ((d.K % 4 == 0) && src_ok(d.a));
    d.b_vec = d.b_pk || ((d.K % 4 == 0) && src_ok(d.b));
  } else if (d.layout == 1) {
    d.a_vec = (d.K % 4 == 0) && src_ok(d.a);
    d.b_vec = (nmem % 4 == 0) && src_ok(d.b);
  } else {
    d.a_vec = (d.M % 4 == 0) && src_ok(d.a);
    d.b_vec = (nmem % 4 == 0) && src_ok(d.b);
  }
}

CglRowSrc rows(const float* p, int ld) {
  CglRowSrc r;
  std::memset(&r, 0, sizeof(r));
  r.p0 = p;
  r.ld = ld;
  r.split = 0x7fffffff;
  return r;
}


}  // namespace

// ------------------------------------------------------------------------------------------
struct cgl_gan {
  cgl_gan_config cfg;
  cgl_gan_buffers bufs;
  WS ws;
  std::vector<CglGemmDesc> gemm;
  std::vector<CglHeadDesc> head;
  std::vector<CglBnBwdDesc> bnb;
  std::vector<CglBnApplyDesc> bna;
  std::vector<Launch> phA, phB;
  hipGraphExec_t gexec[3] = {nullptr, nullptr, nullptr};
  // whole rounds back to back in one graph (cgl_gan_run_graph_rounds): gexec_k[i] holds kRoundGraphs[i] rounds
  static constexpr int kRoundGraphs = 4;
  hipGraphExec_t gexec_k[kRoundGraphs] = {nullptr, nullptr, nullptr, nullptr};
  int gexec_kn[kRoundGraphs] = {0, 0, 0, 0};
  hipStream_t cap = nullptr;   // private capture stream (the legacy default stream cannot capture)
  hipStream_t side = nullptr;  // second stream: the real-row D chain of the first local D step
  CglOpPack pack{};          // the round prologue's operand-packing jobs (none when pack_adam)
  CglOpPack pack_all{};      // every packing job of the plan (cgl_gan_sync_params)
  CglOpPack pack_d{};        // D's packing jobs alone (cgl_gan_sync_params_d)
  bool pack_adam = false;    // G's packed weights written by the G Adam launch (cgl_adam_pack), not the prologue
  bool z_ahead = false;      // z drawn one round ahead by the G Adam launch into ws.znext (plan_z_ahead)
  CglAdamPack adam_pack{};
  CglAdamPack adam_pack_d{};      // D's Adam writing D's packed forward weights (plan_d_pack)
  bool d_pack = false;            // the D forward GEMMs read P(V_j) from ws.dwpk, kept by D's Adam (plan_d_pack)
  std::vector<CglOpPackJob> d_jobs;
  std::vector<CglOpPack> carry;   // packing jobs carried by the forward cgl_bn_apply launches (plan_pack_carriers)
  std::vector<int> pack_need;     // per prologue packing job: the G layer whose forward reads it (INT_MAX: backward)
  unsigned long long* trace = nullptr;   // CGL_GEMM_TRACE diagnostics buffer (kTraceWords per GEMM descriptor)
  int64_t trace_words = 0;
  hipEvent_t ev[2] = {nullptr, nullptr};   // fork (after the prologue), join (before the D-step head)
  bool two_streams = false;
  float* xchg = nullptr;
  int64_t xchg_n = 0;
  int xmode = 0;                     // cgl_gan_exchange_mode: 0 reduce (alpha_scale + all-reduce), 1 gathered
  int ghead = -1;                    // the G-loss head descriptor (its loss_out2 = the exchange slot's loss word)
  std::vector<Launch> phBhead;       // phase B's head under xmode 1: cgl_alpha_combine
  // parameter tensor pointers
  std::vector<TensorRec> gl, dl;
  int64_t run_mean_off[CGL_MAX_LAYERS], run_var_off[CGL_MAX_LAYERS];
  ~cgl_gan() {
    for (auto& g : gexec)
      if (g) (void)hipGraphExecDestroy(g);
    for (auto& g : gexec_k)
      if (g) (void)hipGraphExecDestroy(g);
    if (cap) (void)hipStreamDestroy(cap);
    if (side) (void)hipStreamDestroy(side);
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
    if (trace) (void)hipFree(trace);
  }
};

namespace {

const float* gparam(const cgl_gan* c, int layer, int kind) {
  for (auto& t : c->gl)
    if (t.layer == layer && t.kind == kind) return c->bufs.g_params + t.off;
  return nullptr;
}
float* ggrad(const cgl_gan* c, int layer, int kind) {
  for (auto& t : c->gl)
    if (t.layer == layer && t.kind == kind) return c->bufs.g_grads + t.off;
  return nullptr;
}
const float* dparam(const cgl_gan* c, int layer, int kind) {
  for (auto& t : c->dl)
    if (t.layer == layer && t.kind == kind) return c->bufs.d_params + t.off;
  return nullptr;
}
float* dgrad(const cgl_gan* c, int layer, int kind) {
  for (auto& t : c->dl)
    if (t.layer == layer && t.kind == kind) return c->bufs.d_grads + t.off;
  return nullptr;
}

// BatchNorm1d folded into the neighbouring GEMMs' operand loads instead of the cgl_bn_apply (bit 1:
// forward, a_bn 1) / cgl_bn_bwd (bit 2: backward, a_bn 2) launches.  CGL_BN_FOLD = mask, default 0:
// correct (the MLP GPU suite passes with either bit) but measured slower in the B = 256 round
// (profiles/r03_bn_fold_ab.txt: 0.259 ms separate, 0.270 / 0.269 / 0.281 ms with bit 1 / 2 / both --
// the consumer GEMMs grow by more than the launches they remove: the forward fold's prologue and
// the backward fold's second operand stream, re-read by every column tile)
int bn_fold_mask() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CGL_BN_FOLD");
    v = e ? atoi(e) : 0;
  }
  return v;
}

// Fragment-packed GEMM operands (cgl_pk_off): on by default, CGL_PACK=0 keeps every operand row-major.
bool pack_enabled() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("CGL_PACK");
    v = (e && atoi(e) == 0) ? 0 : 1;
  }
  return v == 1;
}

// Per-descriptor tile arrangement: the plan's measured table (gemm_tile_pick) and the experiment override
// CGL_GEMM_TILE_AT="i:WM,WN,WK[,T];..." (i = the descriptor's index in the plan, as CGL_PLAN_DEBUG prints it;
// read per plan).  Returns true when descriptor i was forced.
bool gemm_tile_at_env(int i, int* o) {
  const char* e = getenv("CGL_GEMM_TILE_AT");
  if (!e) return false;
  const char* q = e;
  while (*q) {
    int di = -1, wm = 0, wn = 0, wk = 0, t = 0, used = 0;
    const int got = sscanf(q, "%d:%d,%d,%d%n,%d%n", &di, &wm, &wn, &wk, &used, &t, &used);
    if (got < 4) break;
    if (di == i && wm * wn * wk == 4) {
      o[0] = wm;
      o[1] = wn;
      o[2] = wk;
      o[3] = (got == 5 && (t == 1 || t == 2)) ? t : 0;
      return true;
    }
    q += used;
    while (*q == ';' || *q == ' ') ++q;
  }
  return false;
}

// XCD blocking of the tile order (cgl_gemm_body): the pm x (8 / pm) slab cut whose L2 working set -- every
// XCD reads A / pm and B pm / 8 -- is smallest, i.e. the least fabric traffic A pn + B pm summed over the
// XCDs (the n-major ranges, pm = 1, read all of A on every XCD).  Measured SLOWER in the B = 256 round
// (0.2666 vs 0.2464 ms, interleaved x3, profiles/r04_xcd_block_ab.txt): the n-major ranges keep a weight
// panel hot in one XCD's L2 while consecutive workgroups sweep the (smaller) activation rows.  Opt-in:
// CGL_XCD_BLOCK=-1 cost model, =1/2/4/8 that pm where the grid allows it; default 0 (n-major ranges).
void choose_xcd(CglGemmDesc& d) {
  static int env = -2;
  if (env == -2) env = getenv("CGL_XCD_BLOCK") ? atoi(getenv("CGL_XCD_BLOCK")) : 0;
  d.xcd_pm = 0;
  if (env == 0 || (long)d.tiles_m * d.tiles_n * (d.ksplit > 1 ? d.ksplit : 1) < 16) return;
  const double A = (double)d.M * d.K, B = (double)(d.N - (d.layout != 0 ? d.b_ones_col : 0)) * d.K;
  double best = 1e300;
  for (int pm : {1, 2, 4, 8}) {
    const int pn = 8 / pm;
    if (pm > d.tiles_m || pn > d.tiles_n) continue;
    if (env > 0 && pm != env) continue;
    const double c = A * pn + B * pm;
    if (c < best * (1.0 - 1e-9)) {
      best = c;
      d.xcd_pm = pm;
    }
  }
}

void set_tiles(CglGemmDesc& d, int wm, int wn, int wk, int t) {
  d.WM = wm;
  d.WN = wn;
  d.WK = wk;
  d.TM = d.TN = t;
  d.tiles_m = (d.M + 32 * t * wm - 1) / (32 * t * wm);
  d.tiles_n = (d.N + 32 * t * wn - 1) / (32 * t * wn);
}

// Measured table over the cost model (tools/tile_search.py, profiles/r04_tile_search.txt): the in-round
// per-descriptor search of the B = 256 round found three problems where two wave rows sharing a column tile
// with a 2-way k split beat the model's 1 x 1 x 4 (the two widest forward GEMMs of G, 512 x 1024 x 512 and
// 512 x 784 x 1024, and G's 1024 x 513 x 256 weight gradient: -0.56 / -0.45 / -0.3 us each, -1.3 us combined
// interleaved x5).  Keyed on the exact problem; everything else keeps the model.
// Round 5 (profiles/r05_tile_search.txt, after D's packed weights): D's 512 x 512 x 256 input gradient (row-major A,
// packed B; the same shape as G2's forward, told apart by its unpacked A) on 1 x 4 x 1, and D0's 512 x 785 x 512
// weight gradient on 2 x 1 x 2: -1.2 / -1.3 us, -2.1 us combined.  Columns: layout, M, N, K, a_pk (-1 any), WM, WN, WK.
bool gemm_tile_pick(const CglGemmDesc& d, int* o) {
  static const int tab[][8] = {{0, 512, 1024, 512, -1, 2, 1, 2}, {0, 512, 784, 1024, -1, 2, 1, 2},
                               {2, 1024, 513, 256, -1, 2, 1, 2}, {0, 512, 512, 256, 0, 1, 4, 1},
                               {2, 512, 785, 512, -1, 2, 1, 2}};
  if (getenv("CGL_TILE_TABLE") && atoi(getenv("CGL_TILE_TABLE")) == 0) return false;
  for (auto& r : tab)
    if (d.layout == r[0] && d.M == r[1] && d.N == r[2] && d.K == r[3] && (r[4] < 0 || d.a_pk == r[4])) {
      o[0] = r[5];
      o[1] = r[6];
      o[2] = r[7];
      return true;
    }
  return false;
}

// Add a grouped GEMM launch built from `descs` (workgroup offsets assigned here).
void push_gemm(cgl_gan* c, std::vector<Launch>& ph, std::vector<CglGemmDesc> descs) {
  Launch L;
  L.kind = K_GEMM;
  L.first = (int)c->gemm.size();
  L.count = (int)descs.size();
  int wg = 0, stage = 0;
  // one block shape per launch (one kernel instantiation): the shape of the largest problem
  int blk = 1;
  double fmax = -1.0;
  for (auto& d : descs) {
    const double f = (double)d.M * d.N * d.K;
    if (f > fmax) {
      fmax = f;
      blk = d.TM;
    }
  }
  int forced[CGL_MAX_LAYERS * 4][4];
  bool isf[CGL_MAX_LAYERS * 4] = {};
  for (int i = 0; i < (int)descs.size() && i < CGL_MAX_LAYERS * 4; ++i) {
    isf[i] = gemm_tile_at_env(L.first + i, forced[i]);
    if (isf[i] && forced[i][3] && descs.size() == 1) blk = forced[i][3];
  }
  for (int i = 0; i < (int)descs.size(); ++i) {
    CglGemmDesc& d = descs[i];
    int pk[3];
    if (i < CGL_MAX_LAYERS * 4 && isf[i] && !d.a_bn)
      set_tiles(d, forced[i][0], forced[i][1], forced[i][2], blk);
    else if (blk == 1 && !d.a_bn && !getenv("CGL_GEMM_TILE") && gemm_tile_pick(d, pk))
      set_tiles(d, pk[0], pk[1], pk[2], 1);
    else if (d.TM != blk)
      choose_tiles(d, 0, blk);
  }
  L.dt = c->cfg.gemm_dtype;
  L.blk = blk;
  long kp = 0;
  unsigned int kc = 0;
  for (auto& d : descs) {
    set_vec(d);
    // split-K: only on the single-stream plan (the partial / ticket regions are per launch), never
    // under an operand transform (its prologue tables are per workgroup)
    d.ksplit = 1;
    if (!c->two_streams && !d.a_bn) {
      choose_ks(d);
      if (d.ksplit > 1 && (kp + cgl_gemm_kpart_floats(d) > kSplitKFloats ||
                           kc + d.tiles_m * d.tiles_n > (unsigned)kSplitKCounters))
        d.ksplit = 1;
      if (d.ksplit > 1) {
        d.kpart = c->ws.kpart + kp;
        d.kcount = c->ws.kcount + kc;
        kp += cgl_gemm_kpart_floats(d);
        kc += d.tiles_m * d.tiles_n;
      }
    }
    d.tab_floats = cgl_gemm_tab_floats(d);
    choose_xcd(d);
    L.abn = std::max(L.abn, d.a_bn);
    d.wg_begin = wg;
    wg += cgl_gemm_wgs(d);
    L.sk = L.sk || d.ksplit > 1;
    const int nalg = d.b_ones_col ? d.N - 1 : d.N;
    L.flops += 2.0 * d.M * (double)nalg * d.K;
    stage = std::max(stage, cgl_gemm_stage_bytes(d));
    c->gemm.push_back(d);
  }
  L.grid = wg;
  L.shmem = stage;
  if (getenv("CGL_PLAN_DEBUG")) {
    for (int q = L.first; q < L.first + L.count; ++q) {
      const CglGemmDesc& d = c->gemm[q];
      fprintf(stderr, "gemm launch %zu: desc %d layout %d M %d N %d K %d WM %d WN %d WK %d TM %d TN %d tiles %dx%d "
              "ks %d grid %d shmem %d blk %d vec %d/%d a_bn %d xcd_pm %d\n", ph.size(), q, d.layout, d.M, d.N, d.K, d.WM,
              d.WN, d.WK, d.TM, d.TN, d.tiles_m, d.tiles_n, d.ksplit, L.grid, L.shmem, L.blk, d.a_vec, d.b_vec, d.a_bn,
              d.xcd_pm);
    }
  }
  ph.push_back(L);
}

void push_head(cgl_gan* c, std::vector<Launch>& ph, const CglHeadDesc& h) {
  Launch L;
  L.kind = K_HEAD;
  L.first = (int)c->head.size();
  L.count = 1;
  L.grid = (h.M + kHeadRows - 1) / kHeadRows;
  c->head.push_back(h);
  ph.push_back(L);
}

void push_bna(cgl_gan* c, std::vector<Launch>& ph, const CglBnApplyDesc& b) {
  Launch L;
  L.kind = K_BNAPPLY;
  L.first = (int)c->bna.size();
  L.count = 1;
  L.grid = (b.F + 63) / 64;
  L.grid_y = (b.bn.mtot + CGL_BNA_ROWS - 1) / CGL_BNA_ROWS;
  c->bna.push_back(b);
  ph.push_back(L);
}

void push_bnb(cgl_gan* c, std::vector<Launch>& ph, const CglBnBwdDesc& b) {
  Launch L;
  L.kind = K_BNBWD;
  L.first = (int)c->bnb.size();
  L.count = 1;
  // features per workgroup (CGL_BNB_FPW = 32 / 16 / 8 / 4, default 8): a narrower slice gives the narrow layers
  // more workgroups (B = 256, F = 256: 8 -> 32 workgroups; 8 measured -6 us/round vs 32, profiles/r03_bnb_ab.txt)
  const int fe = getenv("CGL_BNB_FPW") ? atoi(getenv("CGL_BNB_FPW")) : 8;
  L.blk = (fe == 32 || fe == 16 || fe == 4) ? fe : 8;
  L.grid = (b.F + L.blk - 1) / L.blk;
  c->bnb.push_back(b);
  ph.push_back(L);
}

void push_adam(cgl_gan* c, std::vector<Launch>& ph, float* p, float* g, float* m, float* v, long n,
               const float* ss, const float* bc, int tail, const float* scale = nullptr,
               const unsigned int* found = nullptr) {
  Launch L;
  L.kind = K_ADAM;
  L.adam.p = p;
  L.adam.g = g;
  L.adam.m = m;
  L.adam.v = v;
  L.adam.n = n;
  L.adam.step_size = ss;
  L.adam.bc2sqrt = bc;
  L.adam.b2 = (float)c->cfg.beta2;
  L.adam.w1 = (float)(1.0 - c->cfg.beta1);
  L.adam.w2 = (float)(1.0 - c->cfg.beta2);
  L.adam.eps = (float)c->cfg.adam_eps;
  L.adam.scale = scale;
  L.adam.found = found;
  L.tail = tail;
  L.grid = (int)((n + 255) / 256);
  // four elements per thread (cgl_adam4) when the buffers allow 16-byte access (CGL_ADAM4=0: one per thread)
  const char* e4 = getenv("CGL_ADAM4");
  if (!(e4 && atoi(e4) == 0) && n % 4 == 0 && al16(p) && al16(g) && al16(m) && al16(v)) {
    L.v4 = true;
    L.grid = (int)((n / 4 + 255) / 256);
  }
  ph.push_back(L);
}

// A model's first-layer weight gradient and its Adam as one launch (K_GEMM_ADAM, cgl_gemm_adam): the GEMM
// tiles apply Adam to layer 0's W / b in their epilogue, companion workgroups run Adam over every other
// parameter of the model (which does not depend on this GEMM) and the G Adam's scalar tail.  Applied to
// the last two launches of `ph` when they are that weight gradient and that Adam: G's (the round's last
// two launches) and D's (each local D step's last two).  fp32, no loss scaling (the fused Adam would race
// the GEMM tiles' found flag), layer 0 without BatchNorm.  Correct (bitwise the two launches) but measured
// slower in the B = 256 round, so opt-in: CGL_FUSE_GADAM=1 / CGL_FUSE_DADAM=1 (profiles/r03_fuse_ab.txt:
// the companion Adam floods HBM and the weight-gradient tiles, behind it, end the launch later than the
// two launches did -- G 14.6 -> 15.9 us, D 15.9 -> 19.1 us).
void fuse_wgrad_adam(cgl_gan* c, std::vector<Launch>& ph, int model) {
  const char* var = model == CGL_MODEL_G ? "CGL_FUSE_GADAM" : "CGL_FUSE_DADAM";
  const int env = getenv(var) ? atoi(getenv(var)) : 0;   // read per plan (tests toggle it)
  const cgl_gan_config& cf = c->cfg;
  const cgl_mlp_spec& sp = model == CGL_MODEL_G ? cf.g : cf.d;
  if (!env || cf.loss_scale > 0.f || cf.gemm_dtype != CGL_DTYPE_F32 || sp.bn[0] || ph.size() < 2) return;
  Launch& G = ph[ph.size() - 2];
  Launch& A = ph.back();
  if (G.kind != K_GEMM || G.count != 1 || G.sk || G.abn || A.kind != K_ADAM) return;
  CglGemmDesc& d = c->gemm[G.first];
  const bool gm = model == CGL_MODEL_G;
  float* gw = gm ? ggrad(c, 0, 0) : dgrad(c, 0, 0);
  float* gb = gm ? ggrad(c, 0, 1) : dgrad(c, 0, 1);
  if (d.layout != 2 || d.C != gw || d.bias_out != gb || d.ksplit > 1 || d.a_bn) return;
  float* P = gm ? c->bufs.g_params : c->bufs.d_params;
  float* M = gm ? c->bufs.g_m : c->bufs.d_m;
  float* V = gm ? c->bufs.g_v : c->bufs.d_v;
  if (A.adam.p != P) return;
  // layer 0's tensors lead the flat buffer; the companions cover [off1, n) (layers >= 1, padding incl.)
  int64_t off1 = -1, end0 = 0;
  for (auto& t : gm ? c->gl : c->dl) {
    if (t.layer >= 1 && (off1 < 0 || t.off < off1)) off1 = t.off;
    if (t.layer == 0) end0 = std::max<int64_t>(end0, t.off + (int64_t)t.rows * t.cols);
  }
  if (off1 < end0 || off1 <= 0 || off1 >= A.adam.n) return;
  const int64_t w0 = (gm ? gparam(c, 0, 0) : dparam(c, 0, 0)) - P, b0 = (gm ? gparam(c, 0, 1) : dparam(c, 0, 1)) - P;
  d.ad_p = P + w0;
  d.ad_m = M + w0;
  d.ad_v = V + w0;
  d.ad_pb = P + b0;
  d.ad_mb = M + b0;
  d.ad_vb = V + b0;
  d.ad_ss = A.adam.step_size;
  d.ad_bc = A.adam.bc2sqrt;
  d.ad_b2 = A.adam.b2;
  d.ad_w1 = A.adam.w1;
  d.ad_w2 = A.adam.w2;
  d.ad_eps = A.adam.eps;
  Launch F = G;
  F.kind = K_GEMM_ADAM;
  F.adam = A.adam;
  F.adam.p += off1;
  F.adam.g += off1;
  F.adam.m += off1;
  F.adam.v += off1;
  F.adam.n = A.adam.n - off1;
  F.tail = A.tail;
  F.grid_y = G.grid;                                   // the GEMM's workgroups come first
  F.grid = G.grid + (int)((F.adam.n + CGL_GEMM_THREADS - 1) / CGL_GEMM_THREADS);
  ph.pop_back();
  ph.back() = F;
}

// A head launch followed (same stream, no event between) by a GEMM launch leaves its batch-mean loss reduction
// to that launch: the head workgroups only store their partials (no release, no ticket, no last-arriver
// round trips), and one extra workgroup of the GEMM launch -- its last -- reduces them in the same fixed
// order (cgl_head_finish), so the losses are bitwise those of the ticket path.  The kernel boundary makes the
// partials visible; nothing in the GEMM launch reads the losses.  CGL_HEAD_DEFER=0 keeps the ticket path.
void defer_heads(cgl_gan* c) {
  const int env = getenv("CGL_HEAD_DEFER") ? atoi(getenv("CGL_HEAD_DEFER")) : 1;   // read per plan
  if (!env) return;
  for (std::vector<Launch>* ph : {&c->phA, &c->phB}) {
    for (size_t i = 0; i + 1 < ph->size(); ++i) {
      Launch& H = (*ph)[i];
      Launch& G = (*ph)[i + 1];
      if (H.kind != K_HEAD || G.kind != K_GEMM || H.stream != 0 || G.stream != 0 || H.record_ev >= 0 ||
          G.wait_ev >= 0)
        continue;
      CglGemmDesc& d0 = c->gemm[G.first];
      if (d0.fin_head) continue;
      CglHeadDesc& h = c->head[H.first];
      h.deferred = 1;
      h.nwg = H.grid;
      d0.fin_head = c->ws.head + H.first;
      G.grid += 1;
      G.shmem = std::max(G.shmem, 8 * H.grid);   // the finisher's partials in dynamic LDS
    }
  }
}

// The round prologue and G's first GEMM as one launch (K_GEMM_PRO, cgl_gemm_pro): the GEMM's workgroups
// draw their own rows of z (a_gen; every column tile of a row tile draws the same rows, identical writes),
// the prologue's other blocks ride along.  fp32 plans on one stream; CGL_FUSE_PRO=0 keeps two launches.
void fuse_prologue(cgl_gan* c) {
  const int env = getenv("CGL_FUSE_PRO") ? atoi(getenv("CGL_FUSE_PRO")) : 1;
  std::vector<Launch>& A = c->phA;
  if (!env || c->two_streams || c->cfg.gemm_dtype != CGL_DTYPE_F32 || A.size() < 2) return;
  const Launch& P = A[0];
  const Launch& G = A[1];
  if (P.kind != K_PROLOGUE || G.kind != K_GEMM || G.count != 1 || G.sk || G.abn) return;
  CglGemmDesc& d = c->gemm[G.first];
  // (b_pk: layer 0's packed weights are written by the prologue's pack blocks, which would run in this same
  // launch with no ordering against the GEMM tiles reading them -- keep two launches then)
  if (d.layout != 0 || d.a.p0 != (c->z_ahead ? c->ws.znext : c->bufs.z) || d.a.idx0 || d.a.split != 0x7fffffff ||
      d.a_pk || d.b_pk || d.ksplit > 1)
    return;
  if (c->cfg.gen_z && !c->z_ahead) {
    if (d.M != 2 * c->cfg.batch || d.K != c->cfg.g.dims[0] || d.a.ld != d.K) return;   // the tiles cover every z row
    d.a_gen = 1;
    d.gen_round = &c->ws.st->round;
    d.gen_seed = c->cfg.seed;
    d.gen_n = P.nn;
  }
  Launch F = G;
  F.kind = K_GEMM_PRO;
  F.begin = P.begin;
  F.nptr = P.nptr;
  F.nn = P.nn;
  F.nb_norm = 0;
  F.nb_samp = P.nb_samp;
  F.grid_y = G.grid;
  F.grid = G.grid + (P.grid - P.nb_norm);      // every prologue block but the z draw
  F.record_ev = P.record_ev;
  A.erase(A.begin());
  A[0] = F;
}

// The packing of G's weights moves from the round prologue into the G Adam launch (cgl_adam_pack) when every
// job is a G weight matrix with R, K multiples of 4 (the MNIST / ring / Mix-G specs) and that Adam is a plain
// K_ADAM launch (not CGL_FUSE_GADAM's GEMM-carried form).  The packed copies then always hold the parameters
// the last G Adam wrote; after any other write of G's parameters the caller runs cgl_gan_sync_params (GanStep
// does so whenever the parameter buffer's torch version counter moved).  Bitwise the same rounds
// (tests/test_gpu_pack_adam.py), but measured SLOWER in the B = 256 round (profiles/r05_pack_adam_ab.txt,
// interleaved x3: 0.2433 vs 0.2403 ms): the prologue launch only loses 1.5 us (its packing blocks ran beside
// G's first GEMM on otherwise idle CUs), while the bandwidth-bound G Adam grows 8.2 -> 13.7 us (the 11.6 MB of
// packed writes, and 4 x 4 tiles per thread leave it too few waves).  Opt-in: CGL_PACK_ADAM=1.
// The packing jobs ride in the forward cgl_bn_apply launches (CGL_PACK_CARRY, default on): those launches have
// 4-16 workgroups on a latency chain of ~4.5 us and leave the chip's bandwidth idle, while in the round prologue
// the jobs (G's packed weights P(W) / P(W^T), ~24 MB of traffic) lengthened the launch G's first GEMM rides in.
// A job whose packed copy the forward GEMM of G layer l reads goes to a carrier ahead of that GEMM (carrier
// layer <= l); the backward copies may go to any carrier.  Earliest deadline first, each job to the least loaded
// carrier it may use (bytes), so the carriers' pack blocks stay within their own latency.  Returns false (all
// jobs stay in the prologue) when there is no carrier; a job no carrier may take stays in the prologue.
bool plan_pack_carriers(cgl_gan* c, std::vector<Launch>& A) {
  const char* env = getenv("CGL_PACK_CARRY");
  if ((env && atoi(env) == 0) || c->pack.nj == 0 || (int)c->pack_need.size() != c->pack.nj) return false;
  // carriers: the forward cgl_bn_apply launches (layer = the G layer reading their output) and, for the backward
  // copies only, the deferred loss heads of the D step / G-loss pass (layer INT_MAX - 1: after every G forward)
  std::vector<Launch*> car;
  bool gfwd_done = false;
  for (auto& L : A) {
    if (L.kind == K_BNAPPLY && L.layer >= 0) car.push_back(&L);
    if (L.kind == K_HEAD) gfwd_done = true;
    if (L.kind == K_HEAD && gfwd_done && c->head[L.first].deferred) {
      L.layer = INT_MAX - 1;
      car.push_back(&L);
    }
  }
  if (car.empty()) return false;
  std::vector<int> order(c->pack.nj);
  for (int q = 0; q < c->pack.nj; ++q) order[q] = q;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return c->pack_need[a] < c->pack_need[b]; });
  std::vector<double> load(car.size(), 0.0);
  std::vector<CglOpPack> cp(car.size());
  for (auto& p : cp) std::memset(&p, 0, sizeof(p));
  CglOpPack rest;
  std::memset(&rest, 0, sizeof(rest));
  for (int q : order) {
    const CglOpPackJob& J = c->pack.j[q];
    int best = -1;
    for (int k = 0; k < (int)car.size(); ++k)
      if (car[k]->layer <= c->pack_need[q] && cp[k].nj < CGL_PACK_MAXJ && (best < 0 || load[k] < load[best])) best = k;
    CglOpPack& dst = best >= 0 ? cp[best] : rest;
    CglOpPackJob& D = dst.j[dst.nj++];
    D = J;
    D.blk_begin = dst.blocks;
    dst.blocks += (int)((cgl_pk_floats(J.R, J.K) / 4 + 255) / 256);
    if (best >= 0) load[best] += (double)cgl_pk_floats(J.R, J.K);
  }
  c->carry.clear();
  for (size_t k = 0; k < car.size(); ++k) {
    if (cp[k].nj == 0) continue;
    car[k]->pk = (int)c->carry.size();
    c->carry.push_back(cp[k]);
  }
  c->pack = rest;
  return true;
}

// cgl_adam_pack's 32 x 64 workgroup tiles through LDS (CGL_ADAM_T32, default on; 0: the 4 x 4 thread tiles)
bool adam_t32() {
  const char* e = getenv("CGL_ADAM_T32");
  return !e || atoi(e) != 0;
}

// The packing jobs `jobs` of one model's weight matrices (tensor list tl, parameters at pbase) written by that
// model's Adam launch A (cgl_adam_pack): the tiles of the matrices that carry jobs, element ranges for the rest.
bool build_adam_pack(const CglOpPackJob* jobs, int nj, const std::vector<TensorRec>& tl, const float* pbase,
                     Launch& A, CglAdamPack& out) {
  CglAdamPack pk;
  std::memset(&pk, 0, sizeof(pk));
  std::vector<std::pair<int64_t, int64_t>> spans;
  for (int q = 0; q < nj; ++q) {
    const CglOpPackJob& J = jobs[q];
    const TensorRec* tr = nullptr;
    for (auto& t : tl)
      if (t.kind == 0 && pbase + t.off == J.src) tr = &t;
    if (!tr || tr->rows % 4 || tr->cols % 4 || tr->off % 4) return false;
    // the job's view of W [rows = fo][cols = fi]: forward P(W; fo, fi) or transposed P(W^T; fi, fo)
    const bool fwd = !J.trans && J.R == tr->rows && J.K == tr->cols && J.ld == tr->cols;
    const bool trn = J.trans && J.R == tr->cols && J.K == tr->rows && J.ld == tr->cols;
    if (!fwd && !trn) return false;
    int i = 0;
    while (i < pk.nt && pk.t[i].off != tr->off) ++i;
    if (i == pk.nt) {
      if (pk.nt == CGL_APK_MAXT) return false;
      pk.t[pk.nt++] = CglAdamPackTile{tr->off, tr->rows, tr->cols, nullptr, nullptr, 0, adam_t32() && tr->cols % 8 == 0};
      spans.push_back({tr->off, tr->off + (int64_t)tr->rows * tr->cols});
    }
    (fwd ? pk.t[i].fwd : pk.t[i].trn) = J.dst;
  }
  int blk = 0;
  for (int i = 0; i < pk.nt; ++i) {
    pk.t[i].blk_begin = blk;
    blk += pk.t[i].t32 ? ((pk.t[i].R + 31) / 32) * ((pk.t[i].K + 63) / 64)
                       : (int)(((int64_t)(pk.t[i].R / 4) * (pk.t[i].K / 4) + 255) / 256);
  }
  pk.tile_blocks = blk;
  // element ranges: [0, n) minus the tile tensors
  std::sort(spans.begin(), spans.end());
  int64_t at = 0;
  const int64_t n = A.adam.n;
  auto add = [&](int64_t a0, int64_t a1) {
    if (a1 <= a0) return true;
    if (pk.nr == CGL_APK_MAXR) return false;
    pk.r0[pk.nr] = a0;
    pk.r1[pk.nr] = a1;
    pk.rblk[pk.nr] = blk;
    blk += (int)((a1 - a0 + 255) / 256);
    ++pk.nr;
    return true;
  };
  for (auto& sp : spans) {
    if (!add(at, sp.first)) return false;
    at = sp.second;
  }
  if (!add(at, n)) return false;
  A.adpk = true;
  if (A.adam.znext) {           // the z-ahead blocks come after the parameter blocks
    A.adam.zblk0 = blk;
    blk += (int)((A.adam.nz / 4 + 255) / 256);
  }
  A.grid = blk;
  out = pk;
  return true;
}

bool plan_pack_adam(cgl_gan* c, std::vector<Launch>& ph) {
  const int env = getenv("CGL_PACK_ADAM") ? atoi(getenv("CGL_PACK_ADAM")) : 0;   // read per plan
  c->pack_adam = false;
  if (!env || c->pack.nj == 0 || ph.empty()) return false;
  Launch& A = ph.back();
  if (A.kind != K_ADAM || A.adam.p != c->bufs.g_params) return false;
  if (!build_adam_pack(c->pack.j, c->pack.nj, c->gl, c->bufs.g_params, A, c->adam_pack)) return false;
  c->pack_adam = true;
  return true;
}

// D's hidden-layer weights in the fragment-packed layout for the D forward GEMMs (round 5, CGL_DPACK, default on):
// D's parameters change only in D's Adam launch, which writes the packed copy P(V_j; fo, fi) beside each updated
// matrix (cgl_adam_pack), so every D forward -- the next local D step's and the G-loss pass through the updated
// D -- reads two contiguous 1 KB wave loads per 16-k chunk instead of 32 rows x 64 B.  Decided before the D
// forward descriptors are built (the layers whose matrices qualify); the Adam launches take the jobs later.
bool plan_d_pack(cgl_gan* c) {
  const char* env = getenv("CGL_DPACK");
  const char* fd = getenv("CGL_FUSE_DADAM");
  c->d_pack = false;
  c->d_jobs.clear();
  const int mask = env ? atoi(env) : 3;   // bit 0: forward copies P(V_j), bit 1: transposed copies P(V_j^T)
  if (!mask || (fd && atoi(fd) != 0) || !pack_enabled()) return false;
  const cgl_mlp_spec& d = c->cfg.d;
  for (int j = 0; j + 1 < d.n_layers; ++j) {
    const int fi = d.dims[j], fo = d.dims[j + 1];
    if (fi < 256) continue;
    const float* src = dparam(c, j, 0);
    bool ok = false;
    for (auto& t : c->dl)
      if (t.kind == 0 && c->bufs.d_params + t.off == src) ok = t.rows % 4 == 0 && t.cols % 4 == 0 && t.off % 4 == 0;
    if (!ok || (int)c->d_jobs.size() + 2 > CGL_APK_MAXT) continue;
    CglOpPackJob J;
    std::memset(&J, 0, sizeof(J));
    J.src = src;
    J.ld = fi;
    if (mask & 1) {
      J.dst = c->ws.dwpk[j];
      J.R = fo;
      J.K = fi;
      J.trans = 0;
      c->d_jobs.push_back(J);
    }
    if (mask & 2) {
      J.dst = c->ws.dwtpk[j];
      J.R = fi;
      J.K = fo;
      J.trans = 1;
      c->d_jobs.push_back(J);
    }
  }
  c->d_pack = !c->d_jobs.empty();
  return c->d_pack;
}
// the packed copy of D layer j, or null (the forward GEMM reads V_j row-major)
const float* d_packed(cgl_gan* c, int j, int trans = 0) {
  if (!c->d_pack) return nullptr;
  for (auto& J : c->d_jobs)
    if (J.src == dparam(c, j, 0) && J.trans == trans) return J.dst;
  return nullptr;
}
// The input gradient dX = dY V_j of D layer j ([rows][fo] x [fo][fi]): NT on the packed transpose P(V_j^T) kept by
// D's Adam, or NN on the row-major V_j.  The caller sets the epilogue.
CglGemmDesc d_input_grad(cgl_gan* c, int j, int rows_, const float* dY) {
  const cgl_mlp_spec& d = c->cfg.d;
  const int fi = d.dims[j], fo = d.dims[j + 1];
  const float* pkt = d_packed(c, j, 1);
  CglGemmDesc n = make_gemm(pkt ? 0 : 1, rows_, fi, fo);
  n.a = rows(dY, fo);
  n.a_vec = (fo % 4 == 0);
  if (pkt) {
    n.b = rows(pkt, fo);
    n.b_pk = 1;
    n.b_vec = 1;
    choose_tiles(n);
  } else {
    n.b = rows(dparam(c, j, 0), fi);
  }
  return n;
}

// Each plain GEMM launch (and the prologue-fused one) warms the descriptors of the next GEMM-kind launch in execution order (phase A, phase
// B's head, phase B, then round to the next round's first) into L2 (cgl_gemm_f32's pf argument).  Env
// CGL_GEMM_PF=0 disables it (A/B runs).
void link_gemm_prefetch(cgl_gan* c) {
  const char* e = getenv("CGL_GEMM_PF");
  if (e && atoi(e) == 0) return;
  std::vector<Launch*> order;
  for (std::vector<Launch>* ph : {&c->phA, &c->phBhead, &c->phB})
    for (auto& L : *ph)
      if (L.kind == K_GEMM || L.kind == K_GEMM_PRO || L.kind == K_GEMM_ADAM) order.push_back(&L);
  const int n = (int)order.size();
  for (int i = 0; i < n; ++i) {
    Launch& L = *order[i];
    if ((L.kind != K_GEMM && L.kind != K_GEMM_PRO) || n < 2) continue;
    const Launch& nx = *order[(i + 1) % n];
    L.pf_first = nx.first;
    L.pf_count = nx.kind == K_GEMM_PRO ? 1 : nx.count;
  }
}

int build_plan(cgl_gan* c) {
  const cgl_gan_config& cf = c->cfg;
  const cgl_mlp_spec &g = cf.g, &d = cf.d;
  const int L = g.n_layers, J = d.n_layers;
  const int B = cf.batch, Br = cf.batch_real, Md = Br + B;
  const int img = g.dims[L];
  WS& w = c->ws;
  CglStepState* st = w.st;
  const float sl = cf.slope;
  const bool scaling = cf.loss_scale > 0.f;

  std::vector<Launch>& A = c->phA;
  std::vector<Launch>& Bp = c->phB;

  // ---- z one round ahead (z_ahead): the G Adam launch that ends round r draws round r + 1's z into ws.znext
  // (cgl_adam_zblock; create / reset / cgl_gan_sync_params draw it from the device round state), and G's first
  // GEMM reads it there, copying the rows out to bufs.z (the round's z, read by its weight gradient and the
  // caller).  Before, the workgroups of that GEMM drew their rows of z themselves (a_gen, every column tile of a
  // row tile the same rows: ~3 us of Philox + Box-Muller in front of its k-loop, tools/gemm_trace.py), on the
  // round's critical path; in the Adam launch the draw runs beside the bandwidth-bound parameter update.  Same
  // Philox stream and counter: bitwise the same z.  CGL_Z_AHEAD=0 keeps the in-round draw.
  {
    const int zenv = getenv("CGL_Z_AHEAD") ? atoi(getenv("CGL_Z_AHEAD")) : 1;        // read per plan
    const int genv = getenv("CGL_FUSE_GADAM") ? atoi(getenv("CGL_FUSE_GADAM")) : 0;  // (its Adam rides in a GEMM)
    c->z_ahead = cf.gen_z && zenv && !genv && !c->two_streams;
  }
  // ---- round prologue: per-round scalars, z draw, real-batch sampling (one launch)
  const int* real_idx = c->bufs.real_idx;
  {
    Launch Lp;
    Lp.kind = K_PROLOGUE;
    Lp.begin.st = st;
    Lp.begin.epoch = cf.epoch;
    Lp.begin.lr_g = cf.lr_g;
    Lp.begin.lr_d = cf.lr_d;
    Lp.begin.b1 = cf.beta1;
    Lp.begin.b2 = cf.beta2;
    Lp.begin.scaling = cf.loss_scale > 0.f ? 1 : 0;
    Lp.begin.growth_interval = cf.scale_growth_interval > 0 ? cf.scale_growth_interval : 2000;
    if (cf.gen_z && !c->z_ahead) {
      Lp.nptr = c->bufs.z;
      Lp.nn = (long)2 * B * g.dims[0];
      Lp.nb_norm = (int)((Lp.nn / 4 + 255) / 256);
    }
    if (cf.sample_n > 0) {
      Lp.nb_samp = (cf.epoch * Br + 255) / 256;
      real_idx = w.idx;
    }
    Lp.grid = 1 + Lp.nb_norm + Lp.nb_samp;
    Lp.record_ev = c->two_streams ? 0 : -1;   // fork point of the side stream
    A.push_back(Lp);
  }

  // ---- G forward on [z1; z2] (2B rows; BatchNorm statistics per B-row forward call).  The
  // BatchNorm1d(train) + LeakyReLU of a layer's output is applied by the next layer's GEMM as it
  // loads its A operand (a_bn 1: statistics from this GEMM's per-tile partials, combined in the
  // consumer's prologue), which also writes the activation out for the backward pass; a
  // cgl_bn_apply launch remains for shapes the fold does not cover (and with CGL_BN_FOLD=0).
  CglBnFwd pend;
  std::memset(&pend, 0, sizeof(pend));
  bool pend_on = false;
  for (int l = 0; l < L; ++l) {
    const int fi = g.dims[l], fo = g.dims[l + 1];
    CglGemmDesc e = make_gemm(0, 2 * B, fo, fi);
    if (l + 1 < L && g.bn[l] && B < 64) choose_tiles(e, 1);  // keep producer tiles <= one call
    if (l == 0) {
      e.a = rows(c->z_ahead ? w.znext : c->bufs.z, fi);
      if (c->z_ahead) {           // the round's z rows copied out to bufs.z as the GEMM loads them
        e.a_copy = c->bufs.z;
        e.a_copy_ld = fi;
        e.a_copy_row0 = 0;
      }
    } else {
      e.a = rows(w.gout[l - 1], fi);
    }
    // fragment-packed operands (cgl_pk_off): the weights, packed by the round prologue, and the
    // BatchNorm + LeakyReLU output cgl_bn_apply writes packed beside its row-major copy
    const bool pk_on = pack_enabled();
    if (pk_on && fi >= 256 && c->pack.nj < CGL_PACK_MAXJ) {   // (short-K layers: no gain measured)
      CglOpPackJob& J = c->pack.j[c->pack.nj++];
      J.src = gparam(c, l, 0);
      J.dst = w.wpk[l];
      J.R = fo;
      J.K = fi;
      J.ld = fi;
      J.trans = 0;
      c->pack_need.push_back(l);
      e.b_pk = 1;
    }
    if (pend_on) {
      const int bm = 32 * e.TM * e.WM;
      if ((bn_fold_mask() & 1) && cf.gemm_dtype == CGL_DTYPE_F32 && fi <= CGL_BN_MAXF && B % bm == 0) {
        e.a_bn = 1;
        e.a_bnf = pend;
        e.a_copy = w.gact[l - 1];        // the activation, for the backward pass (both calls' rows)
        e.a_copy_ld = fi;
        e.a_copy_row0 = 0;
      } else {
        CglBnApplyDesc ap;
        std::memset(&ap, 0, sizeof(ap));
        ap.F = fi;
        ap.Y = w.gout[l - 1];
        ap.ld_y = fi;
        ap.act = w.gact[l - 1];
        ap.ld_act = fi;
        ap.bn = pend;
        if (pk_on) {
          ap.act_pk = w.gpk[l - 1];
          e.a_pk = 1;
        }
        push_bna(c, A, ap);
        A.back().layer = l;
        e.a = rows(e.a_pk ? w.gpk[l - 1] : w.gact[l - 1], fi);
      }
      pend_on = false;
    }
    if ((e.a_pk || e.b_pk) && !(l + 1 < L && g.bn[l] && B < 64) && !e.a_bn) choose_tiles(e);
    e.a_vec = (fi % 4 == 0) && al16(e.a.p0);
    e.b = rows(e.b_pk ? w.wpk[l] : gparam(c, l, 0), fi);
    e.b_vec = (fi % 4 == 0);
    e.bias = gparam(c, l, 1);
    if (l == L - 1) {
      e.act = CGL_EPI_ACT_TANH;
    } else if (g.bn[l]) {
      e.act = CGL_EPI_ACT_NONE;
      e.stat_part = w.gpart[l];
      e.stat_gr = B;
    } else {
      e.act = CGL_EPI_ACT_LEAKY;
    }
    e.slope = sl;
    e.C = w.gout[l];
    e.ldc = fo;
    push_gemm(c, A, {e});
    if (l + 1 < L && g.bn[l]) {
      CglBnFwd& bn = pend;
      std::memset(&bn, 0, sizeof(bn));
      bn.part = w.gpart[l];
      // the producer's row-tile height as pushed
      bn.part_bm = 32 * c->gemm.back().TM * c->gemm.back().WM;
      bn.gr = B;
      bn.mtot = 2 * B;
      bn.gamma = gparam(c, l, 2);
      bn.beta = gparam(c, l, 3);
      bn.eps = cf.bn_eps;
      bn.momentum = cf.bn_momentum;
      bn.slope = sl;
      bn.run_mean = c->bufs.g_running + c->run_mean_off[l];
      bn.run_var = c->bufs.g_running + c->run_var_off[l];
      bn.save_mean = w.gmean[l];
      bn.save_invstd = w.ginvstd[l];
      pend_on = true;
    }
  }
  const float* Xd = w.gout[L - 1];
  const float* Xg = w.gout[L - 1] + (int64_t)B * img;

  // ---- local D steps (Worker.train capgan.py:324-341)
  const int C = d.dims[J];
  const float combine = cf.loss == CGL_LOSS_CE2 ? 0.5f : 1.0f;
  // hidden-layer forwards of the D-step input rows [row0, row0 + nrows): part 0 = real rows
  // (through the sampler's index list), part 1 = Xd rows, part 2 = both (one 2-segment GEMM)
  plan_d_pack(c);
  auto d_forward = [&](int ep, int part, int stream, int wait_ev) {
    const int row0 = part == 1 ? Br : 0;
    const int nrows = part == 0 ? Br : part == 1 ? B : Md;
    for (int j = 0; j + 1 < J; ++j) {
      const int fi = d.dims[j], fo = d.dims[j + 1];
      CglGemmDesc e = make_gemm(0, nrows, fo, fi);
      if (j == 0) {
        CglRowSrc r;
        std::memset(&r, 0, sizeof(r));
        r.split = 0x7fffffff;
        r.ld = fi;
        if (part == 1) {
          r.p0 = Xd;
        } else {
          if (real_idx) {
            r.p0 = c->bufs.real;
            r.idx0 = real_idx + (int64_t)ep * Br;
          } else {
            r.p0 = c->bufs.real + (int64_t)ep * Br * fi;
          }
          if (part == 2) {
            r.p1 = Xd;
            r.split = Br;
          }
        }
        e.a = r;
        e.a_vec = (fi % 4 == 0) && al16(c->bufs.real) && al16(Xd);
        e.a_copy = w.R + (int64_t)row0 * fi;
        e.a_copy_ld = fi;
        e.a_copy_row0 = 0;
      } else {
        e.a = rows(w.P[j - 1] + (int64_t)row0 * fi, fi);
        e.a_vec = (fi % 4 == 0);
      }
      e.b = rows(dparam(c, j, 0), fi);
      e.b_vec = (fi % 4 == 0);
      if (const float* pkd = d_packed(c, j)) {
        e.b = rows(pkd, fi);
        e.b_pk = 1;
        e.b_vec = 1;
        choose_tiles(e);
      }
      e.bias = dparam(c, j, 1);
      e.act = CGL_EPI_ACT_LEAKY;
      e.slope = sl;
      e.C = w.P[j] + (int64_t)row0 * fo;
      e.ldc = fo;
      push_gemm(c, A, {e});
      A.back().stream = stream;
      if (j == 0) A.back().wait_ev = wait_ev;
    }
  };
  // the loss head of a part: CE/BCE on the logits, dlogits and the gradient into the last
  // hidden layer; real rows are segment 0 (target valid), Xd rows segment 1 (target fake)
  auto d_head = [&](int ep, int part, int stream, int wait_ev, int record_ev) {
    const int row0 = part == 1 ? Br : 0;
    const int nrows = part == 0 ? Br : part == 1 ? B : Md;
    const int F = d.dims[J - 1];
    CglHeadDesc h;
    std::memset(&h, 0, sizeof(h));
    h.M = nrows;
    h.F = F;
    h.C = C;
    h.loss = cf.loss;
    h.P = w.P[J - 2] + (int64_t)row0 * F;
    h.ldp = F;
    h.W = dparam(c, J - 1, 0);
    h.b = dparam(c, J - 1, 1);
    h.split = part == 0 ? Br : part == 1 ? 0 : Br;
    h.t0 = 1;
    h.t1 = 0;
    h.w0 = combine / Br;
    h.w1 = combine / B;
    h.dlogits = w.dlog + (int64_t)row0 * C;
    h.dP = w.dQ[J - 2] + (int64_t)row0 * F;
    h.lddp = F;
    h.slope = sl;
    h.part = part == 0 ? w.hpart2 : w.hpart;
    h.counter = w.counters + (part == 0 ? 16 : ep);
    if (cf.sample_n > 0 && part != 1) h.n0_dev = &st->real_rows[ep];   // the sampler's short batch
    h.loss_out0 = &st->d_loss_parts[ep][0];
    h.loss_out1 = &st->d_loss_parts[ep][1];
    h.combine = combine;
    h.combine_out = part == 0 ? nullptr : &st->d_loss[ep];
    h.combine_in0 = part == 1 ? &st->d_loss_parts[ep][0] : nullptr;
    h.scale_dev = scaling ? &st->scale[0] : nullptr;
    h.rows_per_wg = kHeadRows;
    push_head(c, A, h);
    A.back().stream = stream;
    A.back().wait_ev = wait_ev;
    A.back().record_ev = record_ev;
  };
  for (int ep = 0; ep < cf.epoch; ++ep) {
    if (ep == 0 && c->two_streams) {
      // the real rows of the first local D step do not depend on G: their forward and loss
      // head run on the side stream concurrently with the G forward (forked after the
      // prologue, joined before the Xd head, whose D_loss combines both segments)
      d_forward(0, 0, 1, 0);
      d_head(0, 0, 1, -1, 1);
      // (the G forward was pushed before; move the side chain in front of it in list order so
      // that a single-stream replay of the list is still a valid order)
      d_forward(0, 1, 0, -1);
      d_head(0, 1, 0, 1, -1);
    } else {
      d_forward(ep, 2, 0, -1);
      d_head(ep, 2, 0, -1, -1);
    }
    // backward: weight grads (TN, + bias column) and input grads (NN, LeakyReLU' mask)
    for (int j = J - 1; j >= 0; --j) {
      std::vector<CglGemmDesc> grp;
      if (j == J - 1) {
        // grad of the output layer: dlogits^T . P[J-2]
        CglGemmDesc t = make_gemm(2, C, d.dims[J - 1] + 1, Md);
        t.a = rows(w.dlog, C);
        t.b = rows(w.P[J - 2], d.dims[J - 1]);
        t.b_ones_col = 1;
        t.C = dgrad(c, J - 1, 0);
        t.ldc = d.dims[J - 1];
        t.bias_out = dgrad(c, J - 1, 1);
        if (scaling) t.inf_flag = &st->found[0];
        grp.push_back(t);
        --j;  // the layer below is handled in the same launch
      }
      {
        const float* in = (j >= 1) ? w.P[j - 1] : w.R;
        CglGemmDesc t = make_gemm(2, d.dims[j + 1], d.dims[j] + 1, Md);
        t.a = rows(w.dQ[j], d.dims[j + 1]);
        t.b = rows(in, d.dims[j]);
        t.b_ones_col = 1;
        t.C = dgrad(c, j, 0);
        t.ldc = d.dims[j];
        t.bias_out = dgrad(c, j, 1);
        if (scaling) t.inf_flag = &st->found[0];
        grp.push_back(t);
      }
      if (j >= 1) {
        CglGemmDesc n = d_input_grad(c, j, Md, w.dQ[j]);
        n.mask_ref = w.P[j - 1];
        n.mask_ld = d.dims[j];
        n.slope = sl;
        n.C = w.dQ[j - 1];
        n.ldc = d.dims[j];
        grp.push_back(n);
      }
      push_gemm(c, A, grp);
    }
    int64_t nd = 0;
    param_layout(d, &nd);
    push_adam(c, A, c->bufs.d_params, c->bufs.d_grads, c->bufs.d_m, c->bufs.d_v, (long)nd,
              &st->d_step_size[ep], &st->d_bc2sqrt[ep], 0, scaling ? &st->scale[0] : nullptr,
              scaling ? &st->found[0] : nullptr);
    if (c->d_pack) {    // D's Adam keeps the packed copies (the D forwards after it read them)
      if (!build_adam_pack(c->d_jobs.data(), (int)c->d_jobs.size(), c->dl, c->bufs.d_params, A.back(),
                           c->adam_pack_d))
        return CGL_E_STATE;   // (plan_d_pack admitted only matrices build_adam_pack accepts)
      A.back().apk_d = 1;
    }
    fuse_wgrad_adam(c, A, CGL_MODEL_D);
  }

  // ---- G loss through the updated D (capgan.py:343-347) and its input gradient
  for (int j = 0; j + 1 < J; ++j) {
    const int fi = d.dims[j], fo = d.dims[j + 1];
    CglGemmDesc e = make_gemm(0, B, fo, fi);
    e.a = rows(j == 0 ? Xg : w.S[j - 1], fi);
    e.a_vec = (fi % 4 == 0);
    e.b = rows(dparam(c, j, 0), fi);
    e.b_vec = (fi % 4 == 0);
    if (const float* pkd = d_packed(c, j)) {
      e.b = rows(pkd, fi);
      e.b_pk = 1;
      e.b_vec = 1;
      choose_tiles(e);
    }
    e.bias = dparam(c, j, 1);
    e.act = CGL_EPI_ACT_LEAKY;
    e.slope = sl;
    e.C = w.S[j];
    e.ldc = fo;
    push_gemm(c, A, {e});
  }
  {
    CglHeadDesc h;
    std::memset(&h, 0, sizeof(h));
    h.M = B;
    h.F = d.dims[J - 1];
    h.C = C;
    h.loss = cf.loss;
    h.P = w.S[J - 2];
    h.ldp = d.dims[J - 1];
    h.W = dparam(c, J - 1, 0);
    h.b = dparam(c, J - 1, 1);
    h.split = B;
    h.t0 = 1;
    h.t1 = 1;
    h.w0 = 1.0f / B;
    h.w1 = 1.0f / B;
    h.dP = w.dS[J - 2];
    h.lddp = d.dims[J - 1];
    h.slope = sl;
    h.part = w.hpart;
    h.counter = w.counters + CGL_MAX_EPOCH;
    h.loss_out0 = &st->g_loss_parts[0];
    c->ghead = (int)c->head.size();
    h.combine = 1.0f;
    h.scale_dev = scaling ? &st->scale[1] : nullptr;
    h.rows_per_wg = kHeadRows;
    push_head(c, A, h);
  }
  for (int j = J - 2; j >= 0; --j) {
    // dS[j-1] = (dS[j] V_j) * leaky'(S[j-1]);  j == 0: dXg = dS[0] V_0, then Tanh'
    CglGemmDesc n = d_input_grad(c, j, B, w.dS[j]);
    n.slope = sl;
    if (j >= 1) {
      n.mask_ref = w.S[j - 1];
      n.mask_ld = d.dims[j];
      n.C = w.dS[j - 1];
      n.ldc = d.dims[j];
    } else {
      n.tanh_ref = Xg;
      n.tanh_ld = img;
      n.C = w.dYL;
      n.ldc = img;
    }
    push_gemm(c, A, {n});
  }

  // ---- G backward (Server.train: F_max.backward() capgan.py:258, on the Xg rows)
  std::vector<Launch>* ph = &A;
  if (cf.exchange_layer == -1) {
    c->xchg = w.dYL;
    c->xchg_n = (int64_t)B * img;
    ph = &Bp;
  }
  // The BatchNorm1d backward of layer l - 1 is folded into the GEMMs around it (a_bn 2): the
  // input-gradient GEMM of layer l stores dy = dA * LeakyReLU'(post) with per-tile {sum dy,
  // sum (y - mean) dy} partials, and layer l - 1's weight- and input-gradient GEMMs apply the
  // BatchNorm backward as they load dy (their k-contiguous problem also writes dgamma / dbeta).
  // Not at the Mix-G exchange point (the all-reduce of dA sits between the two), and a cgl_bn_bwd
  // launch where no input-gradient problem follows (and with CGL_BN_FOLD=0).
  auto gbuf = [&](int l) -> float* { return l == L - 1 ? w.dYL : w.gG[l]; };
  bool gG_packed[CGL_MAX_LAYERS] = {};   // gG[l] has a packed copy (written by cgl_bn_bwd)
  CglBnBwdFold gfold;
  std::memset(&gfold, 0, sizeof(gfold));
  bool gfold_on = false;          // layer l's output gradient is dy in gdA[l] + partials
  for (int l = L - 1; l >= 0; --l) {
    std::vector<CglGemmDesc> grp;
    const int fi = g.dims[l], fo = g.dims[l + 1];
    const float* gA = gfold_on ? w.gdA[l] : gbuf(l);
    if (gfold_on && l == 0) {     // no input-gradient problem to carry the fold: the launch
      CglBnBwdDesc b;             // (dy already masked: no post)
      std::memset(&b, 0, sizeof(b));
      b.M = B;
      b.F = fo;
      b.dA = w.gdA[l];
      b.ld_da = fo;
      b.Y = gfold.y;
      b.ld_y = fo;
      b.mean = gfold.mean;
      b.invstd = gfold.invstd;
      b.gamma = gfold.gamma;
      b.dZ = w.gG[l];
      b.ld_dz = fo;
      b.g_gamma = gfold.g_gamma;
      b.g_beta = gfold.g_beta;
      b.slope = sl;
      if (scaling) b.inf_flag = &st->found[1];
      push_bnb(c, *ph, b);
      gfold_on = false;
      gA = gbuf(l);
    }
    {
      const float* prev;
      if (l == 0)
        prev = c->bufs.z + (int64_t)B * fi;
      else if (g.bn[l - 1])
        prev = w.gact[l - 1] + (int64_t)B * fi;
      else
        prev = w.gout[l - 1] + (int64_t)B * fi;
      CglGemmDesc t = make_gemm(2, fo, fi + 1, B);
      t.a = rows(gA, fo);
      t.b = rows(prev, fi);
      t.b_ones_col = 1;
      t.C = ggrad(c, l, 0);
      t.ldc = fi;
      t.bias_out = ggrad(c, l, 1);
      if (scaling) t.inf_flag = &st->found[1];
      if (gfold_on) {
        t.a_bn = 2;
        t.a_bnb = gfold;
      }
      grp.push_back(t);
    }
    bool fold_next = false;
    if (l >= 1) {
      // dA = dZ W_l: NN on the row-major W, or NT on its packed transpose P(W_l^T) (round prologue)
      // with dZ packed too when cgl_bn_bwd wrote it
      const bool pk = pack_enabled() && !gfold_on && c->pack.nj < CGL_PACK_MAXJ;
      CglGemmDesc n = make_gemm(pk ? 0 : 1, B, fi, fo);
      n.a = rows(gA, fo);
      n.a_vec = (fo % 4 == 0);
      n.b = rows(gparam(c, l, 0), fi);
      if (pk) {
        CglOpPackJob& J = c->pack.j[c->pack.nj++];
        J.src = gparam(c, l, 0);
        J.dst = w.wtpk[l];
        J.R = fi;
        J.K = fo;
        J.ld = fi;
        J.trans = 1;
        c->pack_need.push_back(INT_MAX);
        n.b = rows(w.wtpk[l], fo);
        n.b_pk = 1;
        if (l < L - 1 && gG_packed[l]) {
          n.a = rows(w.gGpk[l], fo);
          n.a_pk = 1;
        }
        choose_tiles(n);
      }
      n.slope = sl;
      n.ldc = fi;
      if (gfold_on) {
        n.a_bn = 2;
        n.a_bnb = gfold;
      }
      if (g.bn[l - 1]) {
        n.C = w.gdA[l - 1];
        fold_next = (bn_fold_mask() & 2) && cf.gemm_dtype == CGL_DTYPE_F32 && cf.exchange_layer != l &&
                    fi <= CGL_BN_MAXF;
        if (fold_next) {
          n.mask_ref = w.gact[l - 1] + (int64_t)B * fi;    // LeakyReLU' of the BatchNorm output
          n.mask_ld = fi;
          n.bnb_part = w.gdpart[l - 1];
          n.bnb_y = w.gout[l - 1] + (int64_t)B * fi;       // the Xg call's BatchNorm input
          n.bnb_ld = fi;
          n.bnb_mean = w.gmean[l - 1] + fi;                // group 1 = the Xg forward call
        }
      } else {
        n.mask_ref = w.gout[l - 1] + (int64_t)B * fi;
        n.mask_ld = fi;
        n.C = w.gG[l - 1];
      }
      grp.push_back(n);
    }
    push_gemm(c, *ph, grp);
    gfold_on = false;
    if (fold_next) {
      gfold.part = w.gdpart[l - 1];
      gfold.tiles = c->gemm.back().tiles_m;
      gfold.F = fi;
      gfold.M = B;
      gfold.mean = w.gmean[l - 1] + fi;
      gfold.invstd = w.ginvstd[l - 1] + fi;
      gfold.gamma = gparam(c, l - 1, 2);
      gfold.g_gamma = ggrad(c, l - 1, 2);
      gfold.g_beta = ggrad(c, l - 1, 3);
      gfold.y = w.gout[l - 1] + (int64_t)B * fi;
      gfold.ldy = fi;
      gfold_on = true;
    }
    if (l >= 1 && cf.exchange_layer == l) {
      c->xchg = g.bn[l - 1] ? w.gdA[l - 1] : w.gG[l - 1];
      c->xchg_n = (int64_t)B * fi;
      ph = &Bp;
    }
    if (l >= 1 && g.bn[l - 1] && !fold_next) {
      CglBnBwdDesc b;
      std::memset(&b, 0, sizeof(b));
      b.M = B;
      b.F = fi;
      b.dA = w.gdA[l - 1];
      b.ld_da = fi;
      b.post = w.gact[l - 1] + (int64_t)B * fi;
      b.ld_post = fi;
      b.Y = w.gout[l - 1] + (int64_t)B * fi;
      b.ld_y = fi;
      b.mean = w.gmean[l - 1] + fi;        // group 1 = the Xg forward call
      b.invstd = w.ginvstd[l - 1] + fi;
      b.gamma = gparam(c, l - 1, 2);
      b.dZ = w.gG[l - 1];
      b.ld_dz = fi;
      b.g_gamma = ggrad(c, l - 1, 2);
      b.g_beta = ggrad(c, l - 1, 3);
      b.slope = sl;
      if (scaling) b.inf_flag = &st->found[1];
      if (pack_enabled() && l - 1 >= 1) {     // the next input-gradient GEMM reads it packed
        b.dZ_pk = w.gGpk[l - 1];
        gG_packed[l - 1] = true;
      }
      push_bnb(c, *ph, b);
    }
  }
  int64_t ng = 0;
  param_layout(g, &ng);
  push_adam(c, *ph, c->bufs.g_params, c->bufs.g_grads, c->bufs.g_m, c->bufs.g_v, (long)ng, &st->g_step_size,
            &st->g_bc2sqrt, 1, scaling ? &st->scale[1] : nullptr, scaling ? &st->found[1] : nullptr);
  if (c->z_ahead) {
    Launch& Ag = ph->back();
    Ag.adam.znext = w.znext;
    Ag.adam.nz = (long)2 * B * g.dims[0];
    Ag.adam.zseed = cf.seed;
    Ag.adam.zblk0 = Ag.grid;
    Ag.grid += (int)((Ag.adam.nz / 4 + 255) / 256);
  }
  fuse_wgrad_adam(c, *ph, CGL_MODEL_G);
  defer_heads(c);      // (before the packing plan: the deferred heads can carry packing jobs)
  // the packing jobs run as the round prologue's last blocks
  {
    int blk = 0;
    for (int q = 0; q < c->pack.nj; ++q) {
      CglOpPackJob& J = c->pack.j[q];
      J.blk_begin = blk;
      blk += (int)((cgl_pk_floats(J.R, J.K) / 4 + 255) / 256);
    }
    c->pack.blocks = blk;
    c->pack_all = c->pack;
    std::memset(&c->pack_d, 0, sizeof(c->pack_d));
    for (auto& J : c->d_jobs) {        // D's packed copies too (sync_params / reset: D written from outside)
      if (c->pack_all.nj == CGL_PACK_MAXJ || c->pack_d.nj == CGL_PACK_MAXJ) return CGL_E_SIZE;
      CglOpPackJob& D = c->pack_all.j[c->pack_all.nj++];
      D = J;
      D.blk_begin = c->pack_all.blocks;
      c->pack_all.blocks += (int)((cgl_pk_floats(J.R, J.K) / 4 + 255) / 256);
      CglOpPackJob& E = c->pack_d.j[c->pack_d.nj++];
      E = J;
      E.blk_begin = c->pack_d.blocks;
      c->pack_d.blocks += (int)((cgl_pk_floats(J.R, J.K) / 4 + 255) / 256);
    }
    if (plan_pack_adam(c, *ph)) {      // the G Adam launch writes the packed copies: no prologue packing
      c->pack.nj = 0;
      c->pack.blocks = 0;
    } else if (plan_pack_carriers(c, A)) {
      blk = c->pack.blocks;            // (the jobs no carrier could take stay in the prologue)
      for (auto& Lq : A)
        if (Lq.kind == K_PROLOGUE) Lq.grid += blk;
    } else {
      for (auto& Lq : A)
        if (Lq.kind == K_PROLOGUE) Lq.grid += blk;
    }
  }
  fuse_prologue(c);
  link_gemm_prefetch(c);
  if ((int)c->gemm.size() > kMaxGemmDescs || (int)c->head.size() > kMaxHeadDescs ||
      (int)c->bnb.size() > kMaxBnDescs || (int)c->bna.size() > kMaxBnDescs)
    return CGL_E_SIZE;
  return CGL_OK;
}


// The prefetch range of a GEMM launch (link_gemm_prefetch) as whole 128-byte lines
CglGemmSel gemm_prefetch(const cgl_gan* c, const Launch& L) {
  CglGemmSel q{};
  if (L.pf_first >= 0) {
    const uintptr_t b = (uintptr_t)(c->ws.gemm + L.pf_first) & ~uintptr_t(127);
    const uintptr_t e = (uintptr_t)(c->ws.gemm + L.pf_first + L.pf_count);
    q.pf = (const int*)b;
    q.pf_lines = std::min(64, (int)((e - b + 127) / 128));
  }
  return q;
}

int exec_launch(cgl_gan* c, const Launch& L, hipStream_t s_main, bool events = true) {
  hipStream_t s = s_main;
  if (events && c->two_streams) {
    if (L.stream == 1) s = c->side;
    if (L.wait_ev >= 0) {
      const hipError_t ew = hipStreamWaitEvent(s, c->ev[L.wait_ev], 0);
      if (ew != hipSuccess) return (int)ew;
    }
  }
  switch (L.kind) {
    case K_GEMM:
      if (L.count > 3) return CGL_E_SIZE;
    {
      CglGemmSel q = gemm_sel(c->gemm.data() + L.first, L.count);
      const CglGemmSel pq = gemm_prefetch(c, L);
      q.pf = pq.pf;
      q.pf_lines = pq.pf_lines;
      launch_gemm(L.blk, L.grid, L.shmem, s, c->ws.gemm + L.first, q, L.sk, L.dt, L.abn);
      break;
    }
    case K_HEAD:
      if (L.pk >= 0)
        klaunch(cgl_head_loss_pk, dim3(L.grid + c->carry[L.pk].blocks), dim3(256), 0, s, c->head[L.first], L.grid,
                c->carry[L.pk]);
      else
        klaunch(cgl_head_loss, dim3(L.grid), dim3(256), 0, s, c->head[L.first]);
      break;
    case K_COMBINE:
      klaunch(cgl_alpha_combine, dim3(L.grid), dim3(256), 0, s, c->ws.st, (const float*)c->ws.gath,
              (long)xchg_slot(c->xchg_n), (long)c->xchg_n, c->xchg);
      break;
    case K_BNAPPLY:
      if (L.pk >= 0)
        klaunch(cgl_bn_apply_pk, dim3(L.grid * L.grid_y + c->carry[L.pk].blocks), dim3(256), 0, s, c->bna[L.first],
                L.grid, L.grid * L.grid_y, c->carry[L.pk]);
      else
        klaunch(cgl_bn_apply, dim3(L.grid, L.grid_y), dim3(256), 0, s, c->bna[L.first]);
      break;
    case K_BNBWD:
      if (L.blk == 16)
        klaunch(cgl_bn_bwd16, dim3(L.grid), dim3(256), 0, s, c->bnb[L.first]);
      else if (L.blk == 8)
        klaunch(cgl_bn_bwd8, dim3(L.grid), dim3(256), 0, s, c->bnb[L.first]);
      else if (L.blk == 4)
        klaunch(cgl_bn_bwd4, dim3(L.grid), dim3(256), 0, s, c->bnb[L.first]);
      else
        klaunch(cgl_bn_bwd, dim3(L.grid), dim3(256), 0, s, c->bnb[L.first]);
      break;
    case K_ADAM:
      if (L.adpk)
        klaunch(cgl_adam_pack, dim3(L.grid), dim3(256), 0, s, L.adam, L.apk_d ? c->adam_pack_d : c->adam_pack,
                c->ws.st, L.tail);
      else if (L.v4)
        klaunch(cgl_adam4, dim3(L.grid), dim3(256), 0, s, L.adam, c->ws.st, L.tail);
      else
        klaunch(cgl_adam, dim3(L.grid), dim3(256), 0, s, L.adam, c->ws.st, L.tail);
      break;
    case K_GEMM_PRO: {     // grid_y = the GEMM's workgroups (fuse_prologue)
      const CglGemmSel pq = gemm_prefetch(c, L);
      if (L.blk == 2)
        klaunch(cgl_gemm_pro<2, 2>, dim3(L.grid), dim3(CGL_GEMM_THREADS), L.shmem, s, c->ws.gemm + L.first, L.grid_y, pq.pf, pq.pf_lines, L.begin, L.nptr,
                                                                      L.nn, c->cfg.seed, c->ws.idx, c->cfg.epoch,
                                                                      c->cfg.batch_real, c->cfg.sample_n,
                                                                      c->cfg.seed ^ 0x5bd1e995ULL, c->pack);
      else
        klaunch(cgl_gemm_pro<1, 1>, dim3(L.grid), dim3(CGL_GEMM_THREADS), L.shmem, s, c->ws.gemm + L.first, L.grid_y, pq.pf, pq.pf_lines, L.begin, L.nptr,
                                                                      L.nn, c->cfg.seed, c->ws.idx, c->cfg.epoch,
                                                                      c->cfg.batch_real, c->cfg.sample_n,
                                                                      c->cfg.seed ^ 0x5bd1e995ULL, c->pack);
      break;
    }
    case K_GEMM_ADAM:      // grid_y = the GEMM's workgroups (fuse_wgrad_adam)
      if (L.blk == 2)
        klaunch(cgl_gemm_adam<2, 2>, dim3(L.grid), dim3(CGL_GEMM_THREADS), L.shmem, s, c->ws.gemm + L.first, L.count, L.grid_y, L.adam,
                                                                       c->ws.st, L.tail);
      else
        klaunch(cgl_gemm_adam<1, 1>, dim3(L.grid), dim3(CGL_GEMM_THREADS), L.shmem, s, c->ws.gemm + L.first, L.count, L.grid_y, L.adam,
                                                                       c->ws.st, L.tail);
      break;
    case K_PROLOGUE:
      klaunch(cgl_round_prologue, dim3(L.grid), dim3(256), 0, s, L.begin, L.nptr, L.nn, c->cfg.seed,
                         L.nb_norm, c->ws.idx, c->cfg.epoch, c->cfg.batch_real, c->cfg.sample_n,
                         c->cfg.seed ^ 0x5bd1e995ULL, c->pack);
      break;
    default:
      return CGL_E_STATE;
  }
  hipError_t e = hipGetLastError();
  if (e == hipSuccess && events && c->two_streams && L.record_ev >= 0) e = hipEventRecord(c->ev[L.record_ev], s);
  return e == hipSuccess ? 0 : (int)e;
}

int run_phase(cgl_gan* c, int phase, hipStream_t s) {
  if (phase == CGL_PHASE_ALL || phase == CGL_PHASE_A)
    for (auto& L : c->phA) {
      const int e = exec_launch(c, L, s);
      if (e) return e;
    }
  if (phase == CGL_PHASE_B && c->xmode == 1)
    for (auto& L : c->phBhead) {
      const int e = exec_launch(c, L, s);
      if (e) return e;
    }
  if (phase == CGL_PHASE_ALL || phase == CGL_PHASE_B)
    for (auto& L : c->phB) {
      const int e = exec_launch(c, L, s);
      if (e) return e;
    }
  return 0;
}

#define HIPCHK(x)                          \
  do {                                     \
    const hipError_t _e = (x);             \
    if (_e != hipSuccess) return (int)_e;  \
  } while (0)

}  // namespace

// ==========================================================================================
static const std::vector<Launch>* phase_list(cgl_gan* c, int phase, int idx, int* local);

extern "C" {

const char* cgl_version(void) { return CGL_VERSION_STR; }

int64_t cgl_gan_param_count(const cgl_gan_config* cfg, int model) {
  if (!cfg || (model != CGL_MODEL_G && model != CGL_MODEL_D)) return CGL_E_ARG;
  int64_t n = 0;
  param_layout(model == CGL_MODEL_G ? cfg->g : cfg->d, &n);
  return n;
}

int cgl_gan_param_tensor(const cgl_gan_config* cfg, int model, int idx, int64_t* offset, int* rows_, int* cols,
                         int* layer, int* kind) {
  if (!cfg || (model != CGL_MODEL_G && model != CGL_MODEL_D)) return CGL_E_ARG;
  auto v = param_layout(model == CGL_MODEL_G ? cfg->g : cfg->d, nullptr);
  if (idx < 0 || idx >= (int)v.size()) return CGL_E_ARG;
  if (offset) *offset = v[idx].off;
  if (rows_) *rows_ = v[idx].rows;
  if (cols) *cols = v[idx].cols;
  if (layer) *layer = v[idx].layer;
  if (kind) *kind = v[idx].kind;
  return CGL_OK;
}

int64_t cgl_gan_running_count(const cgl_gan_config* cfg) {
  if (!cfg) return CGL_E_ARG;
  return running_layout(cfg->g, nullptr, nullptr);
}

int64_t cgl_gan_workspace_bytes(const cgl_gan_config* cfg) {
  const int v = validate(cfg);
  if (v) return v;
  return carve_ws(*cfg, nullptr).total;
}

int cgl_gan_create(const cgl_gan_config* cfg, const cgl_gan_buffers* bufs, cgl_gan** out) {
  CGL_BATCH_GUARD();
  if (!out || !bufs) return CGL_E_ARG;
  *out = nullptr;
  const int v = validate(cfg);
  if (v) return v;
  if (!bufs->g_params || !bufs->g_grads || !bufs->g_m || !bufs->g_v || !bufs->d_params || !bufs->d_grads ||
      !bufs->d_m || !bufs->d_v || !bufs->z || !bufs->real || !bufs->workspace)
    return CGL_E_ARG;
  int has_bn = 0;
  for (int l = 0; l < cfg->g.n_layers; ++l) has_bn |= cfg->g.bn[l];
  if (has_bn && !bufs->g_running) return CGL_E_ARG;
  if (cfg->n_workers > 1 && !bufs->losses_all) return CGL_E_ARG;
  const int64_t need = carve_ws(*cfg, nullptr).total;
  if (bufs->workspace_bytes < need) return CGL_E_SIZE;
  if (!al16(bufs->g_params) || !al16(bufs->d_params) || !al16(bufs->z) || !al16(bufs->workspace))
    return CGL_E_ARG;

  {
    const hipError_t ea = gemm_lds_attr();
    if (ea != hipSuccess) return (int)ea;
  }
  cgl_gan* c = new cgl_gan();
  c->cfg = *cfg;
  {
    // measured slower on MI355X (0.299 vs 0.264 ms per B=256 round: the concurrent chains slow
    // each other and the fork / join add latency), so opt-in only
    const char* e2 = getenv("CGL_TWO_STREAMS");
    c->two_streams = e2 && atoi(e2) != 0 && cfg->d.n_layers >= 2;
  }
  if (c->two_streams) {
    hipError_t es = hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking);
    if (es == hipSuccess) es = hipEventCreateWithFlags(&c->ev[0], hipEventDisableTiming);
    if (es == hipSuccess) es = hipEventCreateWithFlags(&c->ev[1], hipEventDisableTiming);
    if (es != hipSuccess) {
      delete c;
      return (int)es;
    }
  }
  c->bufs = *bufs;
  c->ws = carve_ws(*cfg, bufs->workspace);
  c->gl = param_layout(cfg->g, nullptr);
  c->dl = param_layout(cfg->d, nullptr);
  running_layout(cfg->g, c->run_mean_off, c->run_var_off);
  int e = build_plan(c);
  if (e) {
    delete c;
    return e;
  }
  // the gathered exchange (cgl_gan_exchange_mode 1): the G-loss head also writes the loss into the word after the
  // exchange gradient, and phase B can start with cgl_alpha_combine over the gathered slots
  if (c->xchg && c->ghead >= 0 && c->xchg_n % 4 == 0 && xchg_slot(c->xchg_n) <= xchg_slot_max(c->cfg)) {
    c->head[c->ghead].loss_out2 = c->xchg + c->xchg_n;
    Launch L;
    L.kind = K_COMBINE;
    L.grid = (int)std::min<int64_t>((c->xchg_n / 4 + 255) / 256, 1024);
    c->phBhead.push_back(L);
  }
  // diagnostics: per-workgroup wall-clock stamps of every GEMM problem (only a -DCGL_GEMM_TRACE build writes them)
  if (getenv("CGL_GEMM_TRACE") && atoi(getenv("CGL_GEMM_TRACE")) == 1) {
    c->trace_words = (int64_t)c->gemm.size() * kTraceWords;
    hipError_t te = hipMalloc(&c->trace, c->trace_words * 8);
    if (te == hipSuccess) te = hipMemset(c->trace, 0, c->trace_words * 8);
    if (te != hipSuccess) {
      delete c;
      return (int)te;
    }
    for (size_t q = 0; q < c->gemm.size(); ++q) c->gemm[q].trace = c->trace + q * kTraceWords;
  }
  // upload descriptors, zero counters / state.  The caller's workspace may still have work pending on
  // a non-blocking stream (torch.zeros on a side stream: such streams do not order against the
  // legacy null stream these synchronous copies use), and a fill that lands after the upload zeroes
  // the descriptors: the kernels then dereference null operand pointers.  Drain the device first.
  hipError_t he = hipDeviceSynchronize();
  if (he == hipSuccess)
    he = hipMemcpy(c->ws.gemm, c->gemm.data(), c->gemm.size() * sizeof(CglGemmDesc), hipMemcpyHostToDevice);
  if (he == hipSuccess && !c->head.empty())
    he = hipMemcpy(c->ws.head, c->head.data(), c->head.size() * sizeof(CglHeadDesc), hipMemcpyHostToDevice);
  if (he == hipSuccess && !c->bna.empty())
    he = hipMemcpy(c->ws.bna, c->bna.data(), c->bna.size() * sizeof(CglBnApplyDesc), hipMemcpyHostToDevice);
  if (he == hipSuccess && !c->bnb.empty())
    he = hipMemcpy(c->ws.bnb, c->bnb.data(), c->bnb.size() * sizeof(CglBnBwdDesc), hipMemcpyHostToDevice);
  if (he == hipSuccess) he = hipMemset(c->ws.counters, 0, kCounters * sizeof(unsigned int));
  if (he == hipSuccess) he = hipMemset(c->ws.kcount, 0, kSplitKCounters * sizeof(unsigned int));
  if (he == hipSuccess) he = hipMemset(c->ws.st, 0, sizeof(CglStepState));
  if (he == hipSuccess && c->z_ahead) {   // round 1's z
    const long nz = (long)2 * cfg->batch * cfg->g.dims[0];
    hipLaunchKernelGGL(cgl_znext_draw, dim3((unsigned)((nz / 4 + 255) / 256)), dim3(256), 0, nullptr, c->ws.znext, nz,
                       cfg->seed, (const CglStepState*)c->ws.st);
    he = hipGetLastError();
    if (he == hipSuccess) he = hipDeviceSynchronize();
  }
  if (he == hipSuccess) he = hipDeviceSynchronize();
  if (he != hipSuccess) {
    delete c;
    return (int)he;
  }
  *out = c;
  return CGL_OK;
}

int cgl_gan_destroy(cgl_gan* c) {
  if (!c) return CGL_E_ARG;
  delete c;
  return CGL_OK;
}

int cgl_gan_reset(cgl_gan* c, const float* beta_host, void* stream) {
  CGL_BATCH_GUARD();
  if (!c) return CGL_E_ARG;
  CglStepState h;
  std::memset(&h, 0, sizeof(h));
  h.n_workers = c->cfg.n_workers;
  h.rank = c->cfg.rank;
  h.weighting = c->cfg.weighting;
  h.alpha = 1.f;
  h.scale[0] = h.scale[1] = c->cfg.loss_scale > 0.f ? c->cfg.loss_scale : 1.f;
  for (int i = 0; i < c->cfg.n_workers; ++i) h.beta[i] = beta_host ? beta_host[i] : 1.f / c->cfg.n_workers;
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(hipMemcpyAsync(c->ws.st, &h, sizeof(h), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemsetAsync(c->ws.counters, 0, kCounters * sizeof(unsigned int), s));
  HIPCHK(hipMemsetAsync(c->ws.kcount, 0, kSplitKCounters * sizeof(unsigned int), s));
  if ((c->pack_adam || c->d_pack) && c->pack_all.blocks > 0) {   // the packed weights from the current parameters
    hipLaunchKernelGGL(cgl_pack_all, dim3(c->pack_all.blocks), dim3(256), 0, s, c->pack_all);
    HIPCHK(hipGetLastError());
  }
  if (c->z_ahead) {                                   // the next round's z from the (reset) round counter
    const long nz = (long)2 * c->cfg.batch * c->cfg.g.dims[0];
    hipLaunchKernelGGL(cgl_znext_draw, dim3((unsigned)((nz / 4 + 255) / 256)), dim3(256), 0, s, c->ws.znext, nz,
                       c->cfg.seed, (const CglStepState*)c->ws.st);
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipStreamSynchronize(s));
  return CGL_OK;
}

int64_t cgl_gan_gemm_trace(cgl_gan* c, unsigned long long* host_out, int64_t n) {
  if (!c) return CGL_E_ARG;
  if (!c->trace) return 0;
  if (!host_out || n <= 0) return c->trace_words;
  const int64_t k = std::min<int64_t>(n, c->trace_words);
  hipError_t te = hipDeviceSynchronize();
  if (te == hipSuccess) te = hipMemcpy(host_out, c->trace, k * 8, hipMemcpyDeviceToHost);
  return te == hipSuccess ? k : -(int64_t)te;
}

int cgl_gan_sync_params(cgl_gan* c, void* stream) {
  CGL_BATCH_GUARD();
  if (!c) return CGL_E_ARG;
  if ((c->pack_adam || c->d_pack) && c->pack_all.blocks > 0)   // (the prologue / carriers re-pack G every round)
    hipLaunchKernelGGL(cgl_pack_all, dim3(c->pack_all.blocks), dim3(256), 0, (hipStream_t)stream, c->pack_all);
  if (c->z_ahead) {
    const long nz = (long)2 * c->cfg.batch * c->cfg.g.dims[0];
    hipLaunchKernelGGL(cgl_znext_draw, dim3((unsigned)((nz / 4 + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       c->ws.znext, nz, c->cfg.seed, (const CglStepState*)c->ws.st);
  }
  return (int)hipGetLastError();
}

int cgl_gan_sync_params_d(cgl_gan* c, void* stream) {
  CGL_BATCH_GUARD();
  if (!c) return CGL_E_ARG;
  if (c->d_pack && c->pack_d.blocks > 0)
    hipLaunchKernelGGL(cgl_pack_all, dim3(c->pack_d.blocks), dim3(256), 0, (hipStream_t)stream, c->pack_d);
  return (int)hipGetLastError();
}

int cgl_gan_run(cgl_gan* c, int phase, void* stream) {
  CGL_BATCH_GUARD();
  if (!c || phase < 0 || phase > 2) return CGL_E_ARG;
  return run_phase(c, phase, (hipStream_t)stream);
}

int cgl_gan_run_graph(cgl_gan* c, int phase, void* stream) {
  CGL_BATCH_GUARD();
  if (!c || phase < 0 || phase > 2) return CGL_E_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (!c->gexec[phase]) {
    if (!c->cap) HIPCHK(hipStreamCreateWithFlags(&c->cap, hipStreamNonBlocking));
    HIPCHK(hipStreamSynchronize(s));
    hipGraph_t graph;
    HIPCHK(hipStreamBeginCapture(c->cap, hipStreamCaptureModeThreadLocal));
    const int e = run_phase(c, phase, c->cap);
    hipGraph_t g2;
    const hipError_t ec = hipStreamEndCapture(c->cap, &g2);
    if (e) return e;
    HIPCHK(ec);
    graph = g2;
    hipGraphExec_t ex;
    HIPCHK(hipGraphInstantiate(&ex, graph, nullptr, nullptr, 0));
    (void)hipGraphDestroy(graph);
    c->gexec[phase] = ex;
  }
  HIPCHK(hipGraphLaunch(c->gexec[phase], s));
  return CGL_OK;
}

// the cached graph of `rounds` whole rounds (captured and instantiated on first use; *slot its cache entry)
static int graph_rounds_slot(cgl_gan* c, int rounds, hipStream_t s, int* slot_out) {
  int slot = -1;
  for (int i = 0; i < cgl_gan::kRoundGraphs && slot < 0; ++i)
    if (c->gexec_kn[i] == rounds) slot = i;
  if (slot < 0) {
    // every round reads its per-round values (round counter, z, sampler position, Adam steps, schedules) from the
    // device state the previous round advanced, so `rounds` copies of the round's launch sequence captured back to
    // back are those rounds; the graph launch boundary between rounds (and its completion signal) is gone
    for (int i = 0; i < cgl_gan::kRoundGraphs && slot < 0; ++i)
      if (!c->gexec_k[i]) slot = i;
    if (slot < 0) {                                    // (a small cache: the oldest entry makes room)
      (void)hipGraphExecDestroy(c->gexec_k[0]);
      for (int i = 1; i < cgl_gan::kRoundGraphs; ++i) {
        c->gexec_k[i - 1] = c->gexec_k[i];
        c->gexec_kn[i - 1] = c->gexec_kn[i];
      }
      slot = cgl_gan::kRoundGraphs - 1;
      c->gexec_k[slot] = nullptr;
      c->gexec_kn[slot] = 0;
    }
    if (!c->cap) HIPCHK(hipStreamCreateWithFlags(&c->cap, hipStreamNonBlocking));
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipStreamBeginCapture(c->cap, hipStreamCaptureModeThreadLocal));
    int e = 0;
    for (int r = 0; r < rounds && !e; ++r) e = run_phase(c, CGL_PHASE_ALL, c->cap);
    hipGraph_t g;
    const hipError_t ec = hipStreamEndCapture(c->cap, &g);
    if (e) return e;
    HIPCHK(ec);
    hipGraphExec_t ex;
    const hipError_t ei = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    HIPCHK(ei);
    c->gexec_k[slot] = ex;
    c->gexec_kn[slot] = rounds;
  }
  *slot_out = slot;
  return CGL_OK;
}

int cgl_gan_prepare_graph_rounds(cgl_gan* c, int rounds, void* stream) {
  CGL_BATCH_GUARD();
  if (!c || rounds < 2 || rounds > CGL_MAX_GRAPH_ROUNDS) return CGL_E_ARG;
  int slot;
  return graph_rounds_slot(c, rounds, (hipStream_t)stream, &slot);
}

int cgl_gan_run_graph_rounds(cgl_gan* c, int rounds, void* stream) {
  CGL_BATCH_GUARD();
  if (!c || rounds < 1 || rounds > CGL_MAX_GRAPH_ROUNDS) return CGL_E_ARG;
  if (rounds == 1) return cgl_gan_run_graph(c, CGL_PHASE_ALL, stream);
  int slot;
  const int e = graph_rounds_slot(c, rounds, (hipStream_t)stream, &slot);
  if (e) return e;
  HIPCHK(hipGraphLaunch(c->gexec_k[slot], (hipStream_t)stream));
  return CGL_OK;
}

int cgl_gan_profile(cgl_gan* c, int phase, void* stream, float* us, int n) {
  CGL_BATCH_GUARD();
  if (!c || phase < 0 || phase > 2 || !us) return CGL_E_ARG;
  const int nl = cgl_gan_launch_count(c, phase);
  if (n < nl) return CGL_E_SIZE;
  hipStream_t s = (hipStream_t)stream;
  std::vector<hipEvent_t> ev(2 * nl, nullptr);
  int rc = 0;
  for (auto& e : ev)
    if (!rc) rc = (int)hipEventCreate(&e);
  for (int i = 0; i < nl && !rc; ++i) {
    int li;
    const std::vector<Launch>* v = phase_list(c, phase, i, &li);
    t_prof_ev[0] = ev[2 * i];
    t_prof_ev[1] = ev[2 * i + 1];
    rc = exec_launch(c, (*v)[li], s);
    t_prof_ev[0] = t_prof_ev[1] = nullptr;
  }
  if (!rc) rc = (int)hipStreamSynchronize(s);
  for (int i = 0; i < nl && !rc; ++i) {
    float ms = 0.f;
    rc = (int)hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]);
    us[i] = ms * 1e3f;
  }
  for (auto& e : ev)
    if (e) (void)hipEventDestroy(e);
  return rc;
}

int cgl_gan_alpha_scale(cgl_gan* c, void* stream) {
  CGL_BATCH_GUARD();
  if (!c || !c->xchg) return CGL_E_STATE;
  const long n = (long)c->xchg_n;
  const int grid = (int)std::min<long>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(cgl_alpha_scale, dim3(grid), dim3(256), 0, (hipStream_t)stream, c->ws.st,
                     c->bufs.losses_all, c->xchg, n);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

int cgl_gan_exchange_mode(cgl_gan* c, int mode) {
  CGL_BATCH_GUARD();
  if (!c || (mode != 0 && mode != 1)) return CGL_E_ARG;
  if (mode == 1 && c->phBhead.empty()) return CGL_E_STATE;
  if (mode != c->xmode && c->gexec[CGL_PHASE_B]) {   // phase B's graph changes: re-captured on next use
    (void)hipGraphExecDestroy(c->gexec[CGL_PHASE_B]);
    c->gexec[CGL_PHASE_B] = nullptr;
  }
  c->xmode = mode;
  return CGL_OK;
}

int cgl_gan_gather_buffers(cgl_gan* c, float** send, float** recv, int64_t* slot) {
  if (!c || !send || !recv || !slot) return CGL_E_ARG;
  if (c->phBhead.empty()) return CGL_E_STATE;
  *send = c->xchg;
  *recv = c->ws.gath;
  *slot = xchg_slot(c->xchg_n);
  return CGL_OK;
}

int cgl_gan_exchange_buffer(cgl_gan* c, float** ptr, int64_t* n) {
  if (!c || !ptr || !n) return CGL_E_ARG;
  *ptr = c->xchg;
  *n = c->xchg_n;
  return CGL_OK;
}

int cgl_gan_tensor(cgl_gan* c, int which, float** ptr, int64_t* n) {
  if (!c || !ptr || !n) return CGL_E_ARG;
  const int L = c->cfg.g.n_layers;
  const int B = c->cfg.batch;
  const cgl_mlp_spec& g = c->cfg.g;
  *ptr = nullptr;
  *n = 0;
  if (which == 0) {
    *ptr = c->ws.gout[L - 1];
    *n = (int64_t)2 * B * g.dims[L];
  } else if (which == 1) {
    *ptr = &c->ws.st->g_loss_parts[0];
    *n = 1;
  } else if (which == 2) {
    *ptr = c->ws.dYL;
    *n = (int64_t)B * g.dims[L];
  } else if (which == 3) {                          // device sampler: real-row indices [epoch][Br] (int32)
    *ptr = (float*)c->ws.idx;
    *n = (int64_t)c->cfg.epoch * c->cfg.batch_real;
  } else if (which == 4) {                          // device sampler: real rows per local D step (int32)
    *ptr = (float*)&c->ws.st->real_rows[0];
    *n = c->cfg.epoch;
  } else if (which == 6) {                          // the device round state (CglStepState, raw words)
    *ptr = (float*)c->ws.st;
    *n = (int64_t)(sizeof(CglStepState) / 4);
  } else if (which == 5) {                          // the uploaded GEMM descriptor table (raw words)
    *ptr = (float*)c->ws.gemm;
    *n = (int64_t)(c->gemm.size() * sizeof(CglGemmDesc) / 4);
  } else if (which >= 16 && which < 16 + L) {       // gdA[l]: grad w.r.t. BN+LeakyReLU output (Xg rows)
    *ptr = c->ws.gdA[which - 16];
    *n = (int64_t)B * g.dims[which - 16 + 1];
  } else if (which >= 32 && which < 32 + L) {       // gG[l]: grad w.r.t. Linear output (Xg rows)
    *ptr = c->ws.gG[which - 32];
    *n = (int64_t)B * g.dims[which - 32 + 1];
  } else if (which >= 48 && which < 48 + L) {       // gact[l]: BN+LeakyReLU output (2B rows)
    *ptr = c->ws.gact[which - 48];
    *n = (int64_t)2 * B * g.dims[which - 48 + 1];
  } else if (which >= 64 && which < 64 + L) {       // gout[l]: Linear output (pre-BN) / activation (2B rows)
    *ptr = c->ws.gout[which - 64];
    *n = (int64_t)2 * B * g.dims[which - 64 + 1];
  } else if (which >= 80 && which < 80 + L) {       // saved BN batch mean [2][dims[l+1]] (per forward call)
    *ptr = c->ws.gmean[which - 80];
    *n = (int64_t)2 * g.dims[which - 80 + 1];
  } else if (which >= 96 && which < 96 + L) {       // saved BN invstd [2][dims[l+1]]
    *ptr = c->ws.ginvstd[which - 96];
    *n = (int64_t)2 * g.dims[which - 96 + 1];
  } else if (which >= 112 && which < 112 + c->cfg.d.n_layers - 1) {   // D-step hidden activation P[j]
    const int j = which - 112;                                        // (Br + B rows, last local D step)
    *ptr = c->ws.P[j];
    *n = (int64_t)(c->cfg.batch_real + B) * c->cfg.d.dims[j + 1];
  } else if (which >= 128 && which < 128 + c->cfg.d.n_layers - 1) {   // G-loss pass hidden activation S[j]
    const int j = which - 128;                                        // (B rows, through the updated D)
    *ptr = c->ws.S[j];
    *n = (int64_t)B * c->cfg.d.dims[j + 1];
  } else {
    return CGL_E_ARG;
  }
  if (!*ptr) return CGL_E_ARG;
  return CGL_OK;
}

int cgl_gan_read_stats(cgl_gan* c, cgl_gan_stats* out, void* stream) {
  CGL_BATCH_GUARD();
  if (!c || !out) return CGL_E_ARG;
  CglStepState h;
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(hipMemcpyAsync(&h, c->ws.st, sizeof(h), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  std::memset(out, 0, sizeof(*out));
  out->round = h.round;
  for (int e = 0; e < CGL_MAX_EPOCH; ++e) {
    out->d_loss[e] = h.d_loss[e];
    out->d_real[e] = h.d_loss_parts[e][0];
    out->d_fake[e] = h.d_loss_parts[e][1];
  }
  out->g_loss = h.g_loss_parts[0];
  out->alpha = h.alpha;
  out->F = h.F;
  out->lambda_ = h.lambda;
  out->bn_batches = h.bn_batches;
  for (int m = 0; m < 2; ++m) {
    // after a round and before the next prologue the pending update is not applied yet: report the
    // scale that round used and its own found flag
    out->loss_scale[m] = h.scale[m];
    out->last_skipped[m] = h.scaler_pending ? (h.found[m] != 0u) : h.last_skipped[m];
    out->skipped[m] = h.skipped[m] + (h.scaler_pending && h.found[m] != 0u ? 1 : 0);
  }
  return h.err ? CGL_E_STATE : CGL_OK;   // a fused-BatchNorm rendezvous timed out
}

int cgl_gan_plan_info(cgl_gan* c, int phase, int* n_launches, int* n_gemm, double* flops) {
  if (!c) return CGL_E_ARG;
  int nl = 0, ngm = 0;
  double f = 0;
  auto acc = [&](const std::vector<Launch>& v) {
    for (auto& L : v) {
      ++nl;
      if (L.kind == K_GEMM) {
        ++ngm;
        f += L.flops;
      }
    }
  };
  if (phase == CGL_PHASE_ALL || phase == CGL_PHASE_A) acc(c->phA);
  if (phase == CGL_PHASE_B && c->xmode == 1) acc(c->phBhead);
  if (phase == CGL_PHASE_ALL || phase == CGL_PHASE_B) acc(c->phB);
  if (n_launches) *n_launches = nl;
  if (n_gemm) *n_gemm = ngm;
  if (flops) *flops = f;
  return CGL_OK;
}

static const std::vector<Launch>* phase_list(cgl_gan* c, int phase, int idx, int* local) {
  // CGL_PHASE_ALL enumerates phase A then phase B
  if (phase == CGL_PHASE_A || (phase == CGL_PHASE_ALL && idx < (int)c->phA.size())) {
    *local = idx;
    return &c->phA;
  }
  *local = phase == CGL_PHASE_ALL ? idx - (int)c->phA.size() : idx;
  if (phase == CGL_PHASE_B && c->xmode == 1) {   // phase B under the gathered exchange: the combine head first
    if (*local < (int)c->phBhead.size()) return &c->phBhead;
    *local -= (int)c->phBhead.size();
  }
  return &c->phB;
}

int cgl_gan_launch_count(cgl_gan* c, int phase) {
  if (!c || phase < 0 || phase > 2) return CGL_E_ARG;
  if (phase == CGL_PHASE_A) return (int)c->phA.size();
  if (phase == CGL_PHASE_B) return (int)(c->phB.size() + (c->xmode == 1 ? c->phBhead.size() : 0));
  return (int)(c->phA.size() + c->phB.size());
}

int cgl_gan_launch_info(cgl_gan* c, int phase, int idx, int* kind, double* flops, int* grid) {
  if (!c || phase < 0 || phase > 2 || idx < 0 || idx >= cgl_gan_launch_count(c, phase)) return CGL_E_ARG;
  int li;
  const std::vector<Launch>* v = phase_list(c, phase, idx, &li);
  const Launch& L = (*v)[li];
  if (kind) *kind = (int)L.kind;
  if (flops) *flops = L.flops;
  if (grid) {   // workgroups dispatched (2-D BatchNorm grids flattened, carried packing blocks included)
    *grid = L.kind == K_BNAPPLY ? L.grid * L.grid_y : L.grid;
    if ((L.kind == K_BNAPPLY || L.kind == K_HEAD) && L.pk >= 0) *grid += c->carry[L.pk].blocks;
  }
  return CGL_OK;
}

int cgl_gan_launch_one(cgl_gan* c, int phase, int idx, void* stream) {
  CGL_BATCH_GUARD();
  if (!c || phase < 0 || phase > 2 || idx < 0 || idx >= cgl_gan_launch_count(c, phase)) return CGL_E_ARG;
  int li;
  const std::vector<Launch>* v = phase_list(c, phase, idx, &li);
  return exec_launch(c, (*v)[li], (hipStream_t)stream, false);
}

// ---------------- single ops -------------------------------------------------------------
int64_t cgl_op_workspace_bytes(void) { return 1 << 16; }   // descriptor + BN scratch (F <= 8000)

// One Linear GEMM with its descriptor in the kernel arguments (cgl_gemm_f32_arg): no upload, no host
// synchronisation -- stream-ordered like any torch op, and capturable into a graph.  (The workspace
// arguments of the cgl_linear_* entry points are kept for ABI stability and no longer used.)
static int single_gemm(CglGemmDesc& d, void*, int64_t, hipStream_t s) {
  HIPCHK(gemm_lds_attr());
  d.wg_begin = 0;
  set_vec(d);
  d.ksplit = 1;
  choose_xcd(d);
  const int grid = cgl_gemm_wgs(d), shmem = cgl_gemm_stage_bytes(d);
  if (d.TM == 2)
    klaunch(cgl_gemm_f32_arg<2, 2>, dim3(grid), dim3(CGL_GEMM_THREADS), shmem, s, d);
  else
    klaunch(cgl_gemm_f32_arg<1, 1>, dim3(grid), dim3(CGL_GEMM_THREADS), shmem, s, d);
  return (int)hipGetLastError();
}

int cgl_linear_fwd(const float* X, const float* W, const float* b, float* Y, int M, int N, int K, int act,
                   float slope, void* ws, int64_t wsb, void* stream) {
  CGL_BATCH_GUARD();
  if (!X || !W || !Y || M < 1 || N < 1 || K < 1 || act < 0 || act > 3) return CGL_E_ARG;
  CglGemmDesc d = make_gemm(0, M, N, K);
  d.a = rows(X, K);
  d.a_vec = (K % 4 == 0) && al16(X);
  d.b = rows(W, K);
  d.b_vec = (K % 4 == 0) && al16(W);
  d.bias = b;
  d.act = act;
  d.slope = slope;
  d.C = Y;
  d.ldc = N;
  return single_gemm(d, ws, wsb, (hipStream_t)stream);
}

int cgl_linear_bwd_data(const float* dY, const float* W, float* dX, int M, int N, int K, void* ws, int64_t wsb,
                        void* stream) {
  CGL_BATCH_GUARD();
  if (!dY || !W || !dX || M < 1 || N < 1 || K < 1) return CGL_E_ARG;
  CglGemmDesc d = make_gemm(1, M, K, N);
  d.a = rows(dY, N);
  d.a_vec = (N % 4 == 0) && al16(dY);
  d.b = rows(W, K);
  d.C = dX;
  d.ldc = K;
  return single_gemm(d, ws, wsb, (hipStream_t)stream);
}

int cgl_linear_bwd_weight(const float* dY, const float* X, float* dW, float* db, int M, int N, int K, void* ws,
                          int64_t wsb, void* stream) {
  CGL_BATCH_GUARD();
  if (!dY || !X || !dW || M < 1 || N < 1 || K < 1) return CGL_E_ARG;
  CglGemmDesc d = make_gemm(2, N, K + (db ? 1 : 0), M);
  d.a = rows(dY, N);
  d.b = rows(X, K);
  d.b_ones_col = db ? 1 : 0;
  d.C = dW;
  d.ldc = K;
  d.bias_out = db;
  return single_gemm(d, ws, wsb, (hipStream_t)stream);
}

// Prepared (graph-capturable) Linear GEMMs: the descriptor is written once into caller-owned device
// memory (a synchronous copy at preparation), the launch then only reads it -- no per-call upload
// and no stream synchronisation, unlike the cgl_linear_* ops above.
int64_t cgl_linear_desc_bytes(void) { return (int64_t)((sizeof(CglGemmDesc) + 255) & ~size_t(255)); }

}  // extern "C"
namespace {
int linear_prepare(int op, const float* A, const float* B, const int* b_rows, const float* bias, float* C, float* db,
                   int M, int N, int K, int act, float slope, void* desc, CglLinearLaunch* launch, int c_perm = 0) {
  if (!A || !B || !C || !desc || !launch || M < 1 || N < 1 || K < 1 || act < 0 || act > 3 || !al16(desc))
    return CGL_E_ARG;
  if ((b_rows && op != 0) || (c_perm && op != 2)) return CGL_E_ARG;
  CglGemmDesc d;
  if (op == 0) {            // Y[M][N] = act(X[M][K] W[N][K]^T + b)
    d = make_gemm(0, M, N, K);
    d.a = rows(A, K);
    d.a_vec = (K % 4 == 0) && al16(A);
    d.b = rows(B, K);
    d.b.idx0 = b_rows;      // (gathered W rows: output column n is W row b_rows[n])
    d.b_vec = (K % 4 == 0) && al16(B);
    d.bias = bias;
    d.act = act;
    d.slope = slope;
    d.C = C;
    d.ldc = N;
  } else if (op == 1) {     // dX[M][K] = dY[M][N] W[N][K]
    d = make_gemm(1, M, K, N);
    d.a = rows(A, N);
    d.a_vec = (N % 4 == 0) && al16(A);
    d.b = rows(B, K);
    d.C = C;
    d.ldc = K;
  } else if (op == 2) {     // dW[N][K] = dY[M][N]^T X[M][K], db[N] = column sums of dY
    d = make_gemm(2, N, K + (db ? 1 : 0), M);
    d.a = rows(A, N);
    d.b = rows(B, K);
    d.b_ones_col = db ? 1 : 0;
    d.C = C;
    d.ldc = K;
    d.bias_out = db;
    d.c_perm = c_perm;
  } else {
    return CGL_E_ARG;
  }
  d.wg_begin = 0;
  set_vec(d);
  d.ksplit = 1;
  choose_xcd(d);
  // the descriptor buffer may have been allocated / zeroed on a non-blocking stream that the null
  // stream's copy does not wait for: drain the device so that no pending fill overwrites it
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(desc, &d, sizeof(d), hipMemcpyHostToDevice));
  launch->tm = d.TM;
  launch->grid = cgl_gemm_wgs(d);
  launch->shmem = cgl_gemm_stage_bytes(d);
  launch->flags = 0x100 | d.layout | ((d.a_vec && d.b_vec) ? 4 : 0);   // the kernel's problem selection (CglGemmSel)
  return 0;
}
}  // namespace
extern "C" {

int cgl_linear_prepare(int op, const float* A, const float* B, const float* bias, float* C, float* db, int M, int N,
                       int K, int act, float slope, void* desc, CglLinearLaunch* launch) {
  CGL_BATCH_GUARD();
  return linear_prepare(op, A, B, nullptr, bias, C, db, M, N, K, act, slope, desc, launch);
}

int cgl_linear_prepare_wgrad_nhwc(const float* dY, const float* X, float* dW, float* db, int M, int C, int HW, int K,
                                  void* desc, CglLinearLaunch* launch) {
  CGL_BATCH_GUARD();
  auto lg = [](int v) { return (v >= 2 && v <= (1 << 16) && (v & (v - 1)) == 0) ? __builtin_ctz(v) : -1; };
  const int lc = lg(C), lh = HW == 1 ? 0 : lg(HW);
  if (lc < 0 || lh < 0) return CGL_E_ARG;
  return linear_prepare(2, dY, X, nullptr, nullptr, dW, db, M, C * HW, K, 0, 0.f, desc, launch, lc | lh << 8);
}

int cgl_linear_prepare_gather(const float* X, const float* W, const int* w_rows, const float* bias, float* Y, int M,
                              int N, int K, int act, float slope, void* desc, CglLinearLaunch* launch) {
  CGL_BATCH_GUARD();
  if (!w_rows) return CGL_E_ARG;
  return linear_prepare(0, X, W, w_rows, bias, Y, nullptr, M, N, K, act, slope, desc, launch);
}

int cgl_linear_launch(const void* desc, const CglLinearLaunch* launch, void* stream) {
  CGL_BATCH_GUARD();
  if (!desc || !launch || launch->grid < 1 || (launch->tm != 1 && launch->tm != 2)) return CGL_E_ARG;
  HIPCHK(gemm_lds_attr());
  if (!(launch->flags & 0x100)) return CGL_E_ARG;        // not filled by cgl_linear_prepare
  CglGemmSel sel;
  sel.wg1 = sel.wg2 = INT_MAX;
  sel.meta = launch->flags & 15;
  sel.fin = 0;
  launch_gemm(launch->tm, launch->grid, launch->shmem, (hipStream_t)stream, (const CglGemmDesc*)desc, sel);
  return (int)hipGetLastError();
}

int cgl_act_fwd(const float* X, int64_t n, int act, float slope, float* Y, void* stream) {
  CGL_BATCH_GUARD();
  if (!X || !Y || n < 0 || act < 0 || act > 3) return CGL_E_ARG;
  if (n == 0) return 0;
  const int grid = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(cgl_act_fwd_k, dim3(grid), dim3(256), 0, (hipStream_t)stream, X, (long)n, act, slope, Y);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

int cgl_act_bwd(const float* dY, const float* Y, int64_t n, int act, float slope, float* dX, void* stream) {
  CGL_BATCH_GUARD();
  if (!dY || !Y || !dX || n < 0 || act < 0 || act > 3) return CGL_E_ARG;
  if (n == 0) return 0;
  const int grid = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(cgl_act_bwd_k, dim3(grid), dim3(256), 0, (hipStream_t)stream, dY, Y, (long)n, act, slope, dX);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

int cgl_bn1d_fwd(const float* X, int M, int F, int ldx, const float* gamma, const float* beta, double eps,
                 double momentum, float* running_mean, float* running_var, int train, int act, float slope, float* Y,
                 float* save_mean, float* save_invstd, void* ws, int64_t wsb, void* stream) {
  CGL_BATCH_GUARD();
  if (!X || !Y || !gamma || !beta || M < 1 || F < 1 || ldx < F || (act != 0 && act != 1)) return CGL_E_ARG;
  if (!train && (!running_mean || !running_var)) return CGL_E_ARG;
  if (train && M < 2) return CGL_E_ARG;   // torch: "Expected more than 1 value per channel when training"
  if ((running_mean == nullptr) != (running_var == nullptr)) return CGL_E_ARG;
  if ((save_mean == nullptr) != (save_invstd == nullptr)) return CGL_E_ARG;
  (void)ws;
  (void)wsb;
  hipStream_t s = (hipStream_t)stream;
  CglBn1dDesc d;
  std::memset(&d, 0, sizeof(d));
  d.M = M; d.F = F; d.ldx = ldx; d.train = train; d.act = act;
  d.X = X; d.Y = Y; d.gamma = gamma; d.beta = beta; d.eps = eps; d.momentum = momentum; d.slope = slope;
  d.run_mean = running_mean; d.run_var = running_var; d.save_mean = save_mean; d.save_invstd = save_invstd;
  // the descriptor travels in the kernel arguments: no upload, no host synchronisation
  hipLaunchKernelGGL(cgl_bn1d_fwd_k, dim3((F + 31) / 32), dim3(256), 0, s, d);
  return (int)hipGetLastError();
}

int cgl_bn1d_bwd(const float* dY, const float* Y, const float* X, int M, int F, const float* save_mean,
                 const float* save_invstd, const float* gamma, int act, float slope, float* dX, float* dgamma,
                 float* dbeta, void* ws, int64_t wsb, void* stream) {
  CGL_BATCH_GUARD();
  if (!dY || !X || !save_mean || !save_invstd || !gamma || !dX || M < 1 || F < 1) return CGL_E_ARG;
  if ((act != 0 && act != 1) || (act == 1 && !Y)) return CGL_E_ARG;
  // gamma / beta grads land in the workspace when the caller does not want them
  if ((!dgamma || !dbeta) && (!ws || wsb < 2 * 4 * (int64_t)F || !al16(ws))) return CGL_E_ARG;
  hipStream_t s = (hipStream_t)stream;
  float* scratch = (float*)ws;
  CglBnBwdDesc b;
  std::memset(&b, 0, sizeof(b));
  b.M = M; b.F = F;
  b.dA = dY; b.ld_da = F;
  b.post = act == 1 ? Y : nullptr; b.ld_post = F;
  b.Y = X; b.ld_y = F;
  b.mean = save_mean; b.invstd = save_invstd; b.gamma = gamma;
  b.dZ = dX; b.ld_dz = F;
  b.g_gamma = dgamma ? dgamma : scratch;
  b.g_beta = dbeta ? dbeta : scratch + F;
  b.slope = slope;
  // the descriptor travels in the kernel arguments: no upload, no host synchronisation
  hipLaunchKernelGGL(cgl_bn_bwd_arg, dim3((F + 31) / 32), dim3(256), 0, s, b);
  return (int)hipGetLastError();
}

int cgl_adam_step(float* p, const float* g, float* m, float* v, int64_t n, int step, double lr, double beta1,
                  double beta2, double eps, void* ws, int64_t wsb, void* stream) {
  CGL_BATCH_GUARD();
  if (!p || !g || !m || !v || n < 0 || step < 1) return CGL_E_ARG;
  (void)ws;
  (void)wsb;
  hipStream_t s = (hipStream_t)stream;
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  CglAdamArgs a;
  std::memset(&a, 0, sizeof(a));
  a.p = p;
  a.g = const_cast<float*>(g);   // read only: no loss scale on this entry point
  a.m = m;
  a.v = v;
  a.n = (long)n;
  a.step_size = nullptr;            // the step scalars travel in the kernel arguments (no upload)
  a.bc2sqrt = nullptr;
  a.step_size_v = (float)(lr / bc1);
  a.bc2sqrt_v = (float)std::pow(bc2, 0.5);
  a.b2 = (float)beta2;
  a.w1 = (float)(1.0 - beta1);
  a.w2 = (float)(1.0 - beta2);
  a.eps = (float)eps;
  if (n > 0)
    hipLaunchKernelGGL(cgl_adam, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a, (CglStepState*)nullptr, 0);
  return (int)hipGetLastError();
}

int cgl_normal_fill(float* out, int64_t n, unsigned long long seed, int round, int stream_id, void* stream) {
  CGL_BATCH_GUARD();
  if (!out || n < 0) return CGL_E_ARG;
  if (n == 0) return 0;
  hipLaunchKernelGGL(cgl_normal, dim3((unsigned)((n / 4 + 255) / 256)), dim3(256), 0, (hipStream_t)stream, out,
                     (long)n, seed, round, stream_id);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}

}  // extern "C"

// the conv GAN path (model/lsgan.py) and the evaluation kernels are the second translation unit
// (cgl_conv_tu.hip)
