/* libcglgan_hip -- MI355X-native CGL-GAN worker step, C ABI.
 *
 * The reference (NetworkCommunication/CGL-GAN) has no native code and no FFI: its hot path
 * is the per-worker GAN training step that the Python drivers run through PyTorch ops.
 * Each entry point below replaces one piece of that path; the reference interface it
 * stands in for is cited per function (paths relative to the reference repository root).
 * The Python binding that calls this ABI is cgl-gan_amd/cglgan/_lib.py (ctypes); see
 * INTEGRATION.md for how a reference driver binds it.
 *
 * Conventions: all pointers are device pointers unless stated; `stream` is a hipStream_t
 * passed as void*; every function returns 0 on success, a positive hipError_t value on a
 * HIP failure, or a negative CGL_E* code on an argument error.  The library never
 * allocates device memory: the caller provides every buffer (sizes from the *_count /
 * *_bytes queries) and keeps ownership.
 */
#ifndef CGLGAN_H
#define CGLGAN_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CGL_MAX_LAYERS 8

enum {
  CGL_OK = 0,
  CGL_E_ARG = -1,        /* invalid argument / unsupported shape */
  CGL_E_STATE = -2,      /* call out of order (e.g. graph before create) */
  CGL_E_SIZE = -3        /* a caller buffer is too small */
};

enum { CGL_LOSS_CE2 = 0, CGL_LOSS_BCE = 1 };
enum {
  CGL_WEIGHT_CAPGAN = 0,      /* alpha = softmax(beta * softmax(lambda * l))   capgan.py:247-248        */
  CGL_WEIGHT_MEAN = 1,        /* alpha = 1/N                                   MDGAN/MNIST/mdgan.py:203 */
  CGL_WEIGHT_MIX_SINGLE = 2,  /* alpha = softmax(beta * lambda * l)            mixed-gan.py:276         */
  CGL_WEIGHT_MIX_DOUBLE = 3,  /* alpha = softmax(beta * softmax(lambda * l))   CAPGAN/MNIST/mixed-gan.py:276-278 */
  CGL_WEIGHT_CGLGAN = 4       /* alpha = (beta + softmax(lambda * l)) / 2      CGLGAN/2DMG/main.py:261-264 */
};
enum { CGL_PHASE_ALL = 0, CGL_PHASE_A = 1, CGL_PHASE_B = 2 };
/* Operand type of the step's GEMMs (cgl_gan_config.gemm_dtype).  F32 is the reference arithmetic;
 * F16 / BF16 round each GEMM operand (activations, weights, gradients) to 16 bits as it enters
 * the matrix core and accumulate in fp32 -- autocast-style mixed precision with fp32 master
 * weights, BatchNorm, losses and Adam (BASELINE config 5, "bs512 fp16").  The reference has no
 * 16-bit path, so F16 / BF16 results are outside the fp32 parity band (parity unpinned). */
enum { CGL_DTYPE_F32 = 0, CGL_DTYPE_F16 = 1, CGL_DTYPE_BF16 = 2 };
enum { CGL_MODEL_G = 0, CGL_MODEL_D = 1 };

/* One MLP: n_layers Linear layers, dims[0] -> ... -> dims[n_layers].
 * Hidden layers are Linear -> [BatchNorm1d(eps, momentum) if bn[l]] -> LeakyReLU(slope)
 * (block() of model/mnist_model.py:10-15).  G's last layer is followed by Tanh
 * (model/mnist_model.py:22-23); D's last layer gives 2 logits (CE, :81) or one Sigmoid unit (BCE,
 * MDGAN/MNIST/mnist_model.py:41-42, CGLGAN/2DMG/model.py:63-64). */
typedef struct cgl_mlp_spec {
  int n_layers;
  int dims[CGL_MAX_LAYERS + 1];
  int bn[CGL_MAX_LAYERS];
} cgl_mlp_spec;

typedef struct cgl_gan_config {
  cgl_mlp_spec g, d;
  int batch;            /* B: generated rows per forward call (batch_size, capgan.py:48)          */
  int batch_real;       /* real rows per local D step                                            */
  int epoch;            /* local D steps per round (epoch, capgan.py:50), <= 8                  */
  int loss;             /* CGL_LOSS_*                                                            */
  int weighting;        /* CGL_WEIGHT_*                                                          */
  int n_workers, rank;  /* exchange group of this G replica (1: no exchange)                     */
  int exchange_layer;   /* -1: exchange the G-output gradient (CAPGAN / MDGAN);
                           k > 0: exchange the gradient of G layer k's input (Mix-G trunk/head
                           split: layers >= k are this worker's head, mixed-gan.py:263-281)     */
  double lr_g, lr_d, beta1, beta2, adam_eps;  /* 2e-4, 2e-4, 0.5, 0.999, 1e-8 (capgan.py:52-53,122);
                                                 double like the Python floats torch.optim uses  */
  double bn_eps, bn_momentum;                 /* 0.8, 0.1 (model/mnist_model.py:13)              */
  float slope;                                /* 0.2 (model/mnist_model.py:14)                   */
  unsigned long long seed;                    /* z RNG seed; identical across a server group     */
  int gen_z;            /* 1: the step draws z on device (Philox) each round; 0: caller fills z   */
  int sample_n;         /* >0: in-graph shuffle sampler over sample_n real rows (per-epoch keyed
                           permutation, DataLoader(shuffle=True) capgan.py:282,326-330); 0: the
                           caller provides the round's real rows / indices                      */
  int gemm_dtype;       /* CGL_DTYPE_*: GEMM operand type (0 = fp32, the reference arithmetic)   */
  /* Dynamic loss scaling of the 16-bit GEMM path (torch.cuda.amp.GradScaler semantics, one scaler per
   * model): each model's loss gradient is multiplied by its scale S before the backward pass, the
   * weight gradients are checked for inf / NaN as they are stored and unscaled (x 1/S) in the Adam
   * launch, which skips the step (parameters, moments and torch's step count unchanged) when any was
   * non-finite; between rounds S halves after a skipped step and doubles after
   * scale_growth_interval clean ones.  0 = off (required for fp32).  No reference counterpart (the
   * reference is fp32 only): parity unpinned. */
  float loss_scale;            /* initial S (torch's default init_scale: 65536), 0 = off             */
  int scale_growth_interval;   /* clean steps before S doubles (0: torch's default 2000)             */
} cgl_gan_config;

typedef struct cgl_gan_buffers {
  float* g_params; float* g_grads; float* g_m; float* g_v;  /* flat, cgl_gan_param_count(G)      */
  float* g_running;     /* BatchNorm running_mean/running_var, cgl_gan_running_count()            */
  float* d_params; float* d_grads; float* d_m; float* d_v;  /* flat, cgl_gan_param_count(D)      */
  float* z;             /* [2*batch][g.dims[0]]: z1 (no-grad Xd call) then z2 (Xg call)           */
  const float* real;    /* real rows, row stride g.dims[n_layers]                                 */
  int* real_idx;        /* [epoch*batch_real] gather indices into `real`, or NULL: rows in order  */
  float* losses_all;    /* [n_workers] gathered G losses (exchange), may be NULL when n_workers=1 */
  void* workspace;  int64_t workspace_bytes;   /* cgl_gan_workspace_bytes()                      */
} cgl_gan_buffers;

typedef struct cgl_gan cgl_gan;

/* Host-side scalars of the last round (cgl_gan_read_stats). */
typedef struct cgl_gan_stats {
  int round;
  float d_loss[8];      /* D_loss of each local step  (capgan.py:339)                             */
  float d_real[8], d_fake[8];
  float g_loss;         /* this worker's G loss      (capgan.py:346)                             */
  float alpha;          /* weight of this worker's G-loss gradient                               */
  float F;              /* F_max                     (capgan.py:249)                             */
  float lambda_;        /* Lambda after the round    (capgan.py:259)                             */
  long long bn_batches; /* num_batches_tracked of G's BatchNorm layers                          */
  /* dynamic loss scaling (cgl_gan_config.loss_scale > 0), index 0 = D, 1 = G: the scale the last round
   * used, whether that round's step was skipped (non-finite gradient), skipped steps so far */
  float loss_scale[2];
  int last_skipped[2];
  int skipped[2];
} cgl_gan_stats;

/* ---------------- layout / sizing queries (host only, no device access) ---------------- */
/* Number of floats of the flat parameter buffer of G or D (each tensor 256-byte aligned). */
int64_t cgl_gan_param_count(const cgl_gan_config* cfg, int model);
/* Tensor `idx` (reference state-dict order: Linear weight, bias, then BN weight, bias per layer)
 * of G or D: offset in floats and shape.  Returns 0, or CGL_E_ARG past the last tensor. */
int cgl_gan_param_tensor(const cgl_gan_config* cfg, int model, int idx, int64_t* offset, int* rows, int* cols,
                         int* layer, int* kind /* 0 W, 1 b, 2 BN gamma, 3 BN beta */);
int64_t cgl_gan_running_count(const cgl_gan_config* cfg);
int64_t cgl_gan_workspace_bytes(const cgl_gan_config* cfg);

/* ---------------- fused worker step (replaces Server.train + Worker.train) ---------------- */
/* Validates cfg, plans every launch of a round and writes the launch descriptors into the
 * workspace (capgan.py:211-262 + :316-349, mixed-gan.py:238-292 + :355-392,
 * MDGAN/MNIST/mdgan.py:180-207 + :266-297, CGLGAN/2DMG/main.py:225-278 + :344-375). */
int cgl_gan_create(const cgl_gan_config* cfg, const cgl_gan_buffers* bufs, cgl_gan** out);
int cgl_gan_destroy(cgl_gan* ctx);
/* Zero the round counters / lambda, set the data-size weights beta[n_workers]
 * (capgan.py:149-153) -- host array.  Also refreshes the packed G weight copies (cgl_gan_sync_params). */
int cgl_gan_reset(cgl_gan* ctx, const float* beta_host, void* stream);
/* The GEMMs read fragment-packed copies of the weight matrices: G's are re-packed every round by launches of the
 * round itself (carried by the forward BatchNorm-apply and loss-head launches; by the G Adam launch with
 * CGL_PACK_ADAM=1), D's are written by D's Adam launch as it updates the parameters.  After writing parameters
 * from OUTSIDE the round -- loading a state dict, an initialisation, the Cloud FedAvg (mixed-gan.py:104-124), an
 * E-share or D-swap of D -- call this once (stream-ordered, no host sync) before the next round; cgl_gan_reset
 * does it too.  It also redraws the next round's z (gen_z: the G Adam launch draws round r + 1's z at the end of
 * round r; after the device round state was written from outside -- a resumed run -- call this so that z follows
 * the loaded round counter).  Cheap and idempotent between rounds. */
int cgl_gan_sync_params(cgl_gan* ctx, void* stream);
/* D's packed copies only (after an E-share / D-swap of D's parameters; capturable, no host sync). */
int cgl_gan_sync_params_d(cgl_gan* ctx, void* stream);
/* Diagnostics: with CGL_GEMM_TRACE=1 in the environment at create time and a library built with
 * -DCGL_GEMM_TRACE (tools/build_variant.sh), every GEMM workgroup of the last round stamps the 100 MHz wall
 * clock at kernel entry, body start, k-loop start, first chunk consumed, k-loop end and exit: 8 words per
 * workgroup (6 used), 32768 words per GEMM descriptor in plan order.  Copies min(n, size) words (device-synchronising) and returns the count; returns the buffer size
 * for host_out == null, 0 when tracing is off, a negative HIP error otherwise. */
int64_t cgl_gan_gemm_trace(cgl_gan* ctx, unsigned long long* host_out, int64_t n);
/* Run one round (CGL_PHASE_ALL) or its halves around the exchange: phase A ends with this
 * worker's (unscaled) exchange gradient and G loss; phase B consumes the all-reduced one. */
int cgl_gan_run(cgl_gan* ctx, int phase, void* stream);
/* Same, through a captured hipGraph (captured on first use, replayed after). */
int cgl_gan_run_graph(cgl_gan* ctx, int phase, void* stream);
/* `rounds` complete rounds (phase CGL_PHASE_ALL, 1 <= rounds <= CGL_MAX_GRAPH_ROUNDS) as ONE hipGraph launch: the
 * round's launch sequence captured `rounds` times back to back (captured on first use per count, a few counts
 * cached).  Every round reads its per-round values from the device state the previous one advanced, so this is
 * exactly `rounds` calls of cgl_gan_run_graph(ctx, CGL_PHASE_ALL, stream) without the graph-launch boundary
 * between them (N = 1 worker loops: capgan.py:211-262 + :316-349 repeated over num_communication).  Stats read
 * afterwards describe the last round. */
#define CGL_MAX_GRAPH_ROUNDS 64
int cgl_gan_run_graph_rounds(cgl_gan* ctx, int rounds, void* stream);
/* Capture and instantiate the `rounds`-round graph (2 <= rounds <= CGL_MAX_GRAPH_ROUNDS) without launching it
 * (synchronises `stream` once), so a timed or latency-critical loop never pays the capture. */
int cgl_gan_prepare_graph_rounds(cgl_gan* ctx, int rounds, void* stream);
/* Exchange step: alpha from losses_all (already gathered), then scale this worker's exchange
 * gradient by alpha[rank] in place, ready for an all-reduce(sum). */
int cgl_gan_alpha_scale(cgl_gan* ctx, void* stream);
/* Exchange form.  mode 0 (default, "reduce"): the caller gathers the N losses into losses_all, calls
 * cgl_gan_alpha_scale and all-reduces (sum) the exchange buffer between phase A and phase B.  mode 1
 * ("gathered"): the caller all-gathers each worker's slot (cgl_gan_gather_buffers: [exchange gradient | G loss |
 * padding], slot floats, written by phase A) into the recv buffer [n_workers][slot]; phase B then starts with
 * cgl_alpha_combine -- alpha from the gathered losses, exchange buffer = sum_q alpha_q g_q in rank order
 * (products rounded, bitwise what mode 0 with a rank-ordered sum gives, identical on every rank).  One
 * collective per round instead of two, and alpha runs inside phase B (and its graph).  Changing the mode
 * drops phase B's captured graph.  CGL_E_STATE when the plan has no gathered form. */
int cgl_gan_exchange_mode(cgl_gan* ctx, int mode);
int cgl_gan_gather_buffers(cgl_gan* ctx, float** send, float** recv, int64_t* slot);
/* The exchange gradient buffer (device pointer, float count). */
int cgl_gan_exchange_buffer(cgl_gan* ctx, float** ptr, int64_t* n);
/* Device pointer of an internal tensor: 0 = G output [2B][img] (Xd rows then Xg rows),
 * 1 = own G-loss scalar, 2 = gradient at the G output [B][img] (after Tanh'),
 * 3 / 4 = device sampler (sample_n > 0): the round's real-row indices [epoch][batch_real] / real rows
 * of each local D step [epoch] (int32; a pass ends with a short batch of sample_n mod batch_real rows),
 * 5 = the round's GEMM descriptor table as uploaded by cgl_gan_create (raw 32-bit words),
 * 16+l / 32+l = gradient w.r.t. layer l's activation / Linear output [B][dims[l+1]] (Xg rows),
 * 48+l / 64+l = layer l's BN+LeakyReLU output / Linear output [2B][dims[l+1]],
 * 80+l / 96+l = saved BN batch mean / invstd [2][dims[l+1]],
 * 112+j = D hidden layer j's LeakyReLU output of the (last) local D step [Br+B][d.dims[j+1]],
 * 128+j = the same for the G-loss pass through the updated D [B][d.dims[j+1]]. */
int cgl_gan_tensor(cgl_gan* ctx, int which, float** ptr, int64_t* n);
/* Synchronous copy of the round scalars to the host. */
int cgl_gan_read_stats(cgl_gan* ctx, cgl_gan_stats* out, void* stream);
/* Launch / kernel counts of a phase (for roofline bookkeeping). */
int cgl_gan_plan_info(cgl_gan* ctx, int phase, int* n_launches, int* n_gemm_launches, double* gemm_flops);
/* Per-launch access to the plan (instrumented timing: the caller brackets each launch with
 * events on `stream`).  kind: 0 GEMM, 1 loss head, 2 BN backward, 3 Adam, 4 round prologue
 * (scalars, z RNG, sampler), 5 BN forward apply.  flops = algorithmic GEMM flops (0 for others). */
int cgl_gan_launch_count(cgl_gan* ctx, int phase);
int cgl_gan_launch_info(cgl_gan* ctx, int phase, int idx, int* kind, double* flops, int* grid);
int cgl_gan_launch_one(cgl_gan* ctx, int phase, int idx, void* stream);
/* One round (or phase) issued launch by launch, each launch carrying its own start / stop event pair
 * (the dispatch's begin / end timestamps, the interval rocprofv3's kernel trace reports): us[i] = the
 * device duration of launch i of the phase, in the round's own order and data state (n must be >=
 * cgl_gan_launch_count).  Returns 0 or a negative / HIP error code.  The round
 * advances the training state exactly as cgl_gan_run does. */
int cgl_gan_profile(cgl_gan* ctx, int phase, void* stream, float* us, int n);

/* ---------------- single ops (nn.Module boundary: model/mnist_model.py) ---------------- */
/* Every single op is stream-ordered and asynchronous: its descriptor travels in the kernel arguments
 * (nothing is uploaded, the host never waits), so a sequence of them -- a module's forward + backward --
 * can be captured into a hipGraph / torch.cuda.graph.  The workspace arguments are kept for ABI
 * stability; only cgl_bn1d_bwd uses its workspace (2 F floats for dgamma / dbeta when those are null). */
/* Y[M,N] = act(X[M,K] W[N,K]^T + b)   act: 0 none, 1 LeakyReLU(slope), 2 Tanh, 3 Sigmoid
 * (nn.Linear + the activation module that follows it: model/mnist_model.py:11-14,22-23,77-81,
 * MDGAN/MNIST/mnist_model.py:41-42) */
int cgl_linear_fwd(const float* X, const float* W, const float* b, float* Y, int M, int N, int K, int act,
                   float slope, void* workspace, int64_t ws_bytes, void* stream);
/* dX[M,K] = dY[M,N] W[N,K]   (nn.Linear backward, input grad) */
int cgl_linear_bwd_data(const float* dY, const float* W, float* dX, int M, int N, int K, void* workspace,
                        int64_t ws_bytes, void* stream);
/* dW[N,K] = dY^T X, db[N] = sum_rows dY   (nn.Linear backward, weight/bias grad) */
int cgl_linear_bwd_weight(const float* dY, const float* X, float* dW, float* db, int M, int N, int K,
                          void* workspace, int64_t ws_bytes, void* stream);
/* dX[n] = dY[n] * act'(Y[n]) given the activation OUTPUT Y (LeakyReLU / Tanh / Sigmoid backward) */
int cgl_act_bwd(const float* dY, const float* Y, int64_t n, int act, float slope, float* dX, void* stream);
/* Y[n] = act(X[n])  (a standalone nn.LeakyReLU / nn.Tanh / nn.Sigmoid) */
int cgl_act_fwd(const float* X, int64_t n, int act, float slope, float* Y, void* stream);
/* nn.BatchNorm1d(F, eps, momentum) [+ LeakyReLU(slope) when act == 1] on X[M,F] (row stride ldx):
 * train != 0: batch statistics (biased variance for the output, unbiased for running_var),
 * running stats updated, save_mean / save_invstd written (may be null);
 * train == 0: running statistics (eval mode, capgan.py:204-208).  (model/mnist_model.py:13) */
int cgl_bn1d_fwd(const float* X, int M, int F, int ldx, const float* gamma, const float* beta, double eps,
                 double momentum, float* running_mean, float* running_var, int train, int act, float slope, float* Y,
                 float* save_mean, float* save_invstd, void* workspace, int64_t ws_bytes, void* stream);
/* Train-mode backward of the above: dY = grad of the (activated) output Y (row stride F);
 * act == 1 applies LeakyReLU' from Y.  dX[M,F] = grad of X; dgamma, dbeta (may be null). */
int cgl_bn1d_bwd(const float* dY, const float* Y, const float* X, int M, int F, const float* save_mean,
                 const float* save_invstd, const float* gamma, int act, float slope, float* dX, float* dgamma,
                 float* dbeta, void* workspace, int64_t ws_bytes, void* stream);
/* Flat Adam step t (optim.Adam, torch _single_tensor_adam op order) */
int cgl_adam_step(float* p, const float* g, float* m, float* v, int64_t n, int step, double lr, double beta1,
                  double beta2, double eps, void* workspace, int64_t ws_bytes, void* stream);
/* N(0,1) fill (Philox4x32-10 + Box-Muller); counter = (index, round, stream_id) */
int cgl_normal_fill(float* out, int64_t n, unsigned long long seed, int round, int stream_id, void* stream);
int64_t cgl_op_workspace_bytes(void);

/* Prepared Linear GEMMs (graph-capturable; the fused conv round's nn.Linear layers,
 * model/lsgan.py:8,92): cgl_linear_prepare writes the GEMM descriptor once into caller-owned
 * device memory `desc` (cgl_linear_desc_bytes, 256-byte aligned; synchronous) and fills `launch`;
 * cgl_linear_launch then runs it stream-ordered without any upload or synchronisation, reading the
 * operand pointers given at preparation.  op 0: C[M][N] = act(A[M][K] B[N][K]^T + bias);
 * op 1: C[M][K] = A[M][N] B[N][K]; op 2: C[N][K] = A[M][N]^T B[M][K] and db[N] = column sums of A. */
typedef struct CglLinearLaunch { int tm, grid, shmem, flags; } CglLinearLaunch;   /* filled by cgl_linear_prepare;
                                                                                   flags: the kernel's layout / vector
                                                                                   selection (opaque) */
int64_t cgl_linear_desc_bytes(void);
int cgl_linear_prepare(int op, const float* A, const float* B, const float* bias, float* C, float* db, int M, int N,
                       int K, int act, float slope, void* desc, CglLinearLaunch* launch);
int cgl_linear_launch(const void* desc, const CglLinearLaunch* launch, void* stream);
/* op 0 with gathered weight rows: Y[M][N] = act(X[M][K] W[w_rows[n]][:]^T + bias[n]); w_rows is a device
 * int array of N row indices, each a valid row of W (read at every launch, not checked there).  The conv
 * round's Linear(100, 8192) uses it with the NCHW -> NHWC feature permutation (and the bias packed in the
 * same order), so its output is the NHWC activation of out.view(B, 128, 8, 8) (model/lsgan.py:25)
 * directly, bit for bit the plain op 0 output transposed. */
int cgl_linear_prepare_gather(const float* X, const float* W, const int* w_rows, const float* bias, float* Y, int M,
                              int N, int K, int act, float slope, void* desc, CglLinearLaunch* launch);
/* op 2 on an NHWC activation gradient: dW[c * HW + p][k] = sum_m dY[m][p][c] X[m][k] and db[c * HW + p] =
 * sum_m dY[m][p][c] (db may be null), dY [M][HW][C] -- the reference's NCHW feature order in dW / db, read
 * straight from the NHWC tensor (the GEMM's output rows are permuted at the store); C and HW powers of two
 * (C >= 2).  Bit for bit op 2 on the NCHW transpose of dY. */
int cgl_linear_prepare_wgrad_nhwc(const float* dY, const float* X, float* dW, float* db, int M, int C, int HW, int K,
                                  void* desc, CglLinearLaunch* launch);

/* ---------------- conv GAN ops (model/lsgan.py) ----------------
 * Activations are NHWC (torch channels_last memory of the reference's NCHW tensors); weights are
 * the reference's nn.Conv2d layout [cout][cin][3][3].  No op allocates or synchronises: every
 * launch is stream-ordered (hipGraph-capturable); scratch comes from the caller's workspace. */

/* Workspace bytes for the three conv3x3 ops of one geometry (negative on a bad geometry). */
int64_t cgl_conv3x3_workspace_bytes(int n, int h, int w, int cin, int cout, int stride, int up);
/* Y[n][ho][wo][cout] = drop(act(conv3x3(up2(X)) + bias)): nn.Conv2d(cin, cout, 3, stride, 1)
 * (model/lsgan.py:12,16,19,78), optionally preceded by nn.Upsample(scale_factor=2) (up = 1,
 * stride 1; model/lsgan.py:11,15) and followed by the activation (act: 0 none, 1 LeakyReLU(slope),
 * 2 Tanh, 3 Sigmoid; :14,18,20,78) and the nn.Dropout2d scale drop[n][cout] (may be null; :78).
 * X [n][h][w][cin] is the stored (pre-upsample) input; ho = ((h << up) - 1) / stride + 1. */
int cgl_conv3x3_fwd(const float* X, const float* W, const float* bias, float* Y, int n, int h, int w, int cin,
                    int cout, int stride, int up, int act, float slope, const float* drop, void* workspace,
                    int64_t ws_bytes, void* stream);
/* dX[n][h][w][cin] = gradient of the above w.r.t. X (through the upsample when up = 1), from the
 * gradient dY[n][ho][wo][cout] of the convolution output (autograd of model/lsgan.py's convs). */
int cgl_conv3x3_bwd_data(const float* dY, const float* W, float* dX, int n, int h, int w, int cin, int cout,
                         int stride, int up, void* workspace, int64_t ws_bytes, void* stream);
/* dW[cout][cin][3][3] and db[cout] (may be null) of the convolution from dY and its input X. */
int cgl_conv3x3_bwd_weight(const float* dY, const float* X, float* dW, float* db, int n, int h, int w, int cin,
                           int cout, int stride, int up, void* workspace, int64_t ws_bytes, void* stream);
/* cgl_conv3x3_bwd_weight with X the PRE-BatchNorm map of forward call in_group of in_groups: the convolution's
 * input is LeakyReLU(fmaf(x, scale, shift)) (when in_act == 1; else the affine alone), scale / shift from
 * in_coef [2][in_groups][cin] (cgl_bn2d_fwd_stats_coef's coef), applied in the operand loads -- cgl_eltwise's
 * arithmetic, so the result equals the call on the applied activation bit for bit, and the activation need not
 * be stored.  in_group = -1: X stacks in_groups forward calls of n / in_groups images each (the D step's real
 * and fake calls; at most 2, the wave-unit MFMA weight gradient only).  Supported by the LDS-staged MFMA kernel
 * (the G up-convolutions of model/lsgan.py:11,15), the input-stationary Conv2d(64, 1) of :19 (one call) and
 * the wave-unit MFMA weight gradient (the D convolutions of :78); CGL_E_ARG elsewhere.  With in_act =
 * CGL_EPI_ACT_LEAKY, in_slope must be in (0, 1] (the activation is computed as max(w, w * slope)). */
/* The weight gradient of a one-input-channel conv (the discriminator's Conv2d(1, 16, 3, 2, 1), model/lsgan.py:78)
 * from the gradient at its block's OUTPUT: the LeakyReLU (post = its output) and Dropout2d (drop [n][cout], may be
 * null) backward applied per loaded value, bitwise cgl_act_drop_bwd + cgl_conv3x3_bwd_weight.  Other geometries:
 * CGL_E_ARG. */
int cgl_conv3x3_bwd_weight_actdrop(const float* dY, const float* post, const float* drop, float slope, const float* X,
                                   float* dW, float* db, int n, int h, int w, int cin, int cout, int stride, int up,
                                   void* workspace, int64_t ws_bytes, void* stream);
int cgl_conv3x3_bwd_weight_bnin(const float* dY, const float* X, float* dW, float* db, int n, int h, int w, int cin,
                                int cout, int stride, int up, const float* in_coef, int in_groups, int in_group,
                                int in_act, float in_slope, void* workspace, int64_t ws_bytes, void* stream);

/* Stream-ordered dense layer on the same implicit-GEMM kernels (a 1x1 convolution of M "pixels"):
 * Y[M][N] = act(X[M][K] W[N][K]^T + b) -- nn.Linear of model/lsgan.py:8 (l1, 100 -> 8192) and
 * :92 (adv_layer, 512 -> 1) -- its input gradient dX = dY W and weight gradient dW = dY^T X,
 * db = column sums of dY.  Unlike cgl_linear_* these never synchronise the stream. */
int64_t cgl_dense_workspace_bytes(int M, int K, int N);
int cgl_dense_fwd(const float* X, const float* W, const float* b, float* Y, int M, int K, int N, int act, float slope,
                  void* workspace, int64_t ws_bytes, void* stream);
int cgl_dense_bwd_data(const float* dY, const float* W, float* dX, int M, int K, int N, void* workspace,
                       int64_t ws_bytes, void* stream);
int cgl_dense_bwd_weight(const float* dY, const float* X, float* dW, float* db, int M, int K, int N, void* workspace,
                         int64_t ws_bytes, void* stream);

/* Pre-packed weight operands.  The ops above re-pack W into the MFMA operand layout on every call
 * (one extra launch each); a training round instead packs every layer of a model, forward (dir 0)
 * and input-gradient (dir 1) operands, in one launch after each parameter update (the reference
 * has no equivalent: autograd reads W directly, model/lsgan.py:12-99) and passes the packed
 * operand Wp to the *_packed ops.  ks = 3 (conv3x3 geometry) or 1 (dense: h = w = 1, stride 1,
 * up 0, cin = K, cout = N).  Packed layout depends only on (h, w, cin, cout, stride, up, ks, dir). */
typedef struct CglConvPackJob {
  const float* W;            /* [cout][cin][ks][ks], the reference's layout */
  float* Wp;                 /* cgl_conv_packed_floats(...) floats, 16-byte aligned */
  int h, w, cin, cout, stride, up, ks, dir;
} CglConvPackJob;
int64_t cgl_conv_packed_floats(int h, int w, int cin, int cout, int stride, int up, int ks, int dir);
/* all jobs in one launch (at most 48 packed problems: a forward up-conv is 4, a stride-2
 * input gradient 4, everything else 1) */
int cgl_conv_pack_multi(int njobs, const CglConvPackJob* jobs, void* stream);
/* Launch batching (the conv round's start, the D step's two loss heads): between cgl_conv_batch_begin(stream) and
 * cgl_conv_batch_end(stream), at most one each of cgl_conv_pack_multi, cgl_dropout2d_masks(_dev),
 * cgl_normal_fill_dev and cgl_sample_rows_dev, and up to two cgl_adv_loss, on that stream validate and record
 * their arguments instead of launching; _end launches them as ONE kernel (their blocks by range).  The batched
 * calls must not depend on each other (they read and write disjoint buffers).  Same results as the separate
 * launches; one launch floor instead of several.  While a batch is open on the calling thread every OTHER
 * entry point that launches or synchronises (convs, BatchNorm, gather, the MLP step and single ops, ...)
 * returns CGL_E_STATE without launching, so nothing can run ahead of the deferred calls. */
int cgl_conv_batch_begin(void* stream);
int cgl_conv_batch_end(void* stream);
/* Deferred weight-gradient reductions (the conv round's D and G backward): between cgl_conv_wgrad_defer_begin()
 * and cgl_conv_wgrad_defer_end(stream), these calls on the calling thread record their last step instead of
 * launching it: cgl_conv3x3_bwd_weight(_bnin / _actdrop) launch their MFMA kernel and record the fixed-order split
 * reduction (up to 4) or the single-input-channel kernel's finish (one); a column-sum bias gradient (no bias
 * column in the reduction) runs its column-sum pass at once and records its finish, as cgl_colsum_finalize does
 * (up to 3 finishes); one cgl_dense_bwd_weight with N = 1 records its whole launch.  _end launches every recorded
 * step as ONE kernel on that stream.  Bitwise the separate launches.  Each recorded step reads its partials or
 * inputs when _end runs, so every deferred weight gradient needs its OWN workspace, and those buffers and the
 * dense inputs stay untouched until _end; dW / db are written at _end.  A call the batch cannot take (a fifth
 * reduction, a fourth finish) launches at once, as outside a batch.  Other entry points are unaffected.
 * Returns CGL_E_STATE for a nested begin or an end without begin. */
int cgl_conv_wgrad_defer_begin(void);
int cgl_conv_wgrad_defer_end(void* stream);
/* Inside an open deferral: the deferred launch also carries the round's device counters (one extra block, after
 * every other deferred step of the launch): *snap = counters[snap_index], then counters[0 .. n) += v, n <= 64 --
 * cgl_counters_add folded into the G backward's deferred launch of the conv round (its G Adam then reads the
 * completed-step count from *snap).  Nothing else in the launch may read the counters.  At most once per
 * deferral (CGL_E_STATE otherwise, or outside a deferral). */
int cgl_conv_wgrad_defer_counters(int* counters, int n, int v, int* snap, int snap_index);
int cgl_conv3x3_fwd_packed(const float* X, const float* Wp, const float* bias, float* Y, int n, int h, int w, int cin,
                           int cout, int stride, int up, int act, float slope, const float* drop, void* workspace,
                           int64_t ws_bytes, void* stream);
/* W (may be null) is read only by the one-output-channel stride-1 input gradient, which uses the
 * unpacked weights */
int cgl_conv3x3_bwd_data_packed(const float* dY, const float* W, const float* Wp, float* dX, int n, int h, int w,
                                int cin, int cout, int stride, int up, void* workspace, int64_t ws_bytes,
                                void* stream);
/* The forward with the next BatchNorm2d's statistics computed in its epilogue (no separate pass
 * over Y): part [groups * chunks][cout][2] doubles = {sum, M2 about the chunk mean} of every 32-row
 * chunk of the stored output (after act / drop), the chunks of forward call g contiguous.
 * cgl_conv3x3_stat_chunks gives the chunk count (groups * chunks; 0 when unsupported: cout < 32 or a
 * call's rows not whole 32-row chunks).  Consumed by cgl_bn2d_fwd_stats (R = 32). */
int64_t cgl_conv3x3_stat_chunks(int n, int h, int w, int cin, int cout, int stride, int up, int groups);
int cgl_conv3x3_fwd_packed_stats(const float* X, const float* Wp, const float* bias, float* Y, int n, int h, int w,
                                 int cin, int cout, int stride, int up, int act, float slope, const float* drop,
                                 int groups, double* part, const int* nvalid, void* workspace, int64_t ws_bytes,
                                 void* stream);
/* cgl_conv3x3_fwd_packed(_stats) whose input X is the PRE-BatchNorm2d map of a bn2d_fwd_stats_coef call: the
 * BatchNorm (+ LeakyReLU when in_act = CGL_EPI_ACT_LEAKY) is applied to each operand as it is loaded, from
 * in_coef = [2][in_groups][cin] (scale, then shift, per forward call of n / in_groups images), with
 * cgl_eltwise's arithmetic -- the convolution of the applied activation, without that map being written
 * (model/lsgan.py:15-17,20-22: BatchNorm2d -> LeakyReLU -> Upsample -> Conv2d).  part may be null (no
 * statistics of the output).  With in_act = CGL_EPI_ACT_LEAKY, in_slope must be in (0, 1] (CGL_E_ARG otherwise:
 * the activation is computed as max(w, w * slope), the select's value for every input only then). */
int cgl_conv3x3_fwd_packed_bnin(const float* X, const float* Wp, const float* bias, float* Y, int n, int h, int w,
                                int cin, int cout, int stride, int up, int act, float slope, const float* drop,
                                int groups, double* part, const float* in_coef, int in_groups, int in_act,
                                float in_slope, const int* nvalid, void* ws, int64_t wsb, void* stream);
/* The input gradient with the previous BatchNorm2d's backward statistics computed in its epilogue:
 * part [groups * chunks][cin][2] = {sum g, sum g (x - mean)} per 32-row chunk of dX, g = dX (*
 * leaky'(bn_post) when bn_post is given), x = bn_x (the BatchNorm input) and mean = bn_mean
 * [groups][cin] (the saved per-call mean), all at dX's positions.  Consumed by cgl_bn2d_bwd_stats.
 * bn_post_coef (may be null; then bn_post): leaky' from the sign of fmaf(bn_x, scale, shift) with scale =
 * bn_post_coef[c], shift = bn_post_coef[bn_post_coef_ld + c] (cgl_bn2d_bwd's post_coef; groups == 1).
 * cgl_conv3x3_bwd_stat_chunks: chunk count (0: unsupported). */
int64_t cgl_conv3x3_bwd_stat_chunks(int n, int h, int w, int cin, int cout, int stride, int up, int groups);
int cgl_conv3x3_bwd_data_packed_stats(const float* dY, const float* Wp, float* dX, int n, int h, int w, int cin,
                                      int cout, int stride, int up, int groups, double* part, const float* bn_x,
                                      const float* bn_post, const float* bn_post_coef, int bn_post_coef_ld,
                                      const float* bn_mean, float slope, void* workspace, int64_t ws_bytes,
                                      void* stream);
/* The same statistics from the vector one-output-channel input gradient (Conv2d(64, 1, 3, 1, 1) + Tanh,
 * model/lsgan.py:19-20; raw OIHW W, no packing) -- per 128-ROW chunk, the chunking of cgl_bn2d_bwd, so
 * cgl_bn2d_bwd_stats(R = 128) gives bitwise cgl_bn2d_bwd's result on the stored dX (the channel reduction
 * launch saved) whenever cgl_bn2d_bwd itself reduces in 128-row chunks, i.e. a call of at least 64 such chunks
 * ((n / groups) h w >= 8192; smaller calls get 32-64-row chunks there, a different but equally valid order).
 * Other geometries: CGL_E_ARG.  (n / groups) h w must be a multiple of 128. */
int cgl_conv3x3_bwd_data_stats(const float* dY, const float* W, float* dX, int n, int h, int w, int cin, int cout,
                               int stride, int up, int groups, double* part, const float* bn_x, const float* bn_post,
                               const float* bn_post_coef, int bn_post_coef_ld, const float* bn_mean, float slope,
                               void* workspace, int64_t ws_bytes, void* stream);
int cgl_dense_fwd_packed(const float* X, const float* Wp, const float* b, float* Y, int M, int K, int N, int act,
                         float slope, void* workspace, int64_t ws_bytes, void* stream);
int cgl_dense_bwd_data_packed(const float* dY, const float* Wp, float* dX, int M, int K, int N, void* workspace,
                              int64_t ws_bytes, void* stream);

/* nn.BatchNorm2d(C, eps, momentum) [+ LeakyReLU(slope) when act == 1] on NHWC X[n][hw][C]
 * (model/lsgan.py:13,17,80).  `groups` independent forward calls are stacked along n (statistics
 * per group, running stats updated group by group in call order); save_mean / save_invstd are
 * [groups][C] (may be null).  train == 0: running statistics (eval).
 * nvalid (device int32, may be null; here and in the _stats / bwd variants, cgl_conv3x3_fwd_packed_stats
 * and cgl_adv_loss): the first call is a SHORT batch -- only its first *nvalid images are data (the D step's
 * real call on DataLoader's short final batch, capgan.py:282,326-331); the rest of the call's n / groups
 * images are padding: left out of its statistics (mean / variance over *nvalid images, running variance
 * unbiased over them) and given a zero input gradient in the backward. */
int64_t cgl_bn2d_workspace_bytes(int n, int hw, int C, int groups);
int cgl_bn2d_fwd(const float* X, int n, int hw, int C, int groups, const float* gamma, const float* beta, double eps,
                 double momentum, float* running_mean, float* running_var, int train, int act, float slope, float* Y,
                 float* save_mean, float* save_invstd, const int* nvalid, void* workspace, int64_t ws_bytes,
                 void* stream);
/* Train-mode backward: dY is the gradient of the BatchNorm output, or of LeakyReLU(output) when
 * `post` (that activation's output) is given.  The result is optionally multiplied by
 * LeakyReLU'(post_out) and the Dropout2d scale drop[n][C] (the Conv -> LeakyReLU -> Dropout2d ->
 * BatchNorm2d block of model/lsgan.py:78-80, backward in one pass).  dgamma / dbeta may be null. */
/* cgl_bn2d_fwd (train) from statistics partials already computed (R rows per chunk, the layout of
 * cgl_conv3x3_fwd_packed_stats): finalize + apply only.  scratch (may be null; 256-byte aligned,
 * cgl_bn2d_stats_scratch_bytes, ZEROED ONCE by the caller and kept per BatchNorm layer): lets a call
 * with more than 1024 chunks per forward call finalize in parallel slices (monotonic tickets). */
int64_t cgl_bn2d_stats_scratch_bytes(int C, int groups);
int cgl_bn2d_fwd_stats(const double* part, int R, const float* X, int n, int hw, int C, int groups, const float* gamma,
                       const float* beta, double eps, double momentum, float* running_mean, float* running_var,
                       int act, float slope, float* Y, float* save_mean, float* save_invstd, void* scratch,
                       const int* nvalid, void* workspace, int64_t ws_bytes, void* stream);
/* cgl_bn2d_fwd_stats, also writing the per-(group, channel) scale / shift it applies into coef
 * ([2][groups][C]: scale, then shift; may be null) and applying them to images [apply_img0, n) only:
 * the rest is left for a consumer that folds the BatchNorm into its operand load
 * (cgl_conv3x3_fwd_packed_bnin). */
int cgl_bn2d_fwd_stats_coef(const double* part, int R, const float* X, int n, int hw, int C, int groups,
                            const float* gamma, const float* beta, double eps, double momentum, float* running_mean,
                            float* running_var, int act, float slope, float* Y, float* save_mean, float* save_invstd,
                            void* scratch, float* coef, int apply_img0, const int* nvalid, void* ws, int64_t wsb,
                            void* stream);
/* 1 when cgl_conv3x3_bwd_weight(_bnin) of this geometry computes its bias gradient by column sums of dY in
 * 256-row chunks (cgl_bn2d_bwd_stats colsum_part + cgl_colsum_finalize reproduce it bitwise), 0 when its
 * reduction carries a bias column (or the single-input-channel kernel sums it); < 0 for a bad geometry. */
int cgl_conv3x3_bias_by_colsum(int n, int h, int w, int cin, int cout, int stride, int up);
/* cgl_bn2d_bwd from backward partials already computed (cgl_conv3x3_bwd_data_packed_stats, R = 32).
 * colsum_part (may be null): also the column sums of dX per 256-row chunk, double [n hw / 256][C][2] ({sum, 0}),
 * in the order of the channel reduction cgl_conv3x3_bwd_weight runs for a bias gradient without a bias column --
 * cgl_colsum_finalize(colsum_part, n hw / 256, C, db) then gives that bias gradient bitwise, without the pass
 * over dX.  Needs C % 4 == 0, 256 % (C / 4) == 0, n hw % 256 == 0. */
int cgl_bn2d_bwd_stats(const double* part, int R, const float* dY, const float* post, const float* X, int n, int hw,
                       int C, int groups, const float* save_mean, const float* save_invstd, const float* gamma,
                       float slope, const float* post_out, const float* drop, float* dX, float* dgamma, float* dbeta,
                       const float* post_coef, int post_coef_ld, const int* nvalid, double* colsum_part,
                       void* workspace, int64_t ws_bytes, void* stream);
/* post_coef (may be null; then post as above): instead of reading post, take LeakyReLU'(post) from the sign of
 * the forward's fmaf(X, scale, shift) with scale = post_coef[c], shift = post_coef[post_coef_ld + c] (the coef a
 * cgl_bn2d_fwd_stats_coef call kept; its group g of G: post_coef = coef + g C, post_coef_ld = G C).  The forward
 * wrote post = LeakyReLU(that value), so the two signs agree bit for bit and post's bytes are not read.
 * Requires post == null and groups == 1 (one forward call's rows). */
int cgl_bn2d_bwd(const float* dY, const float* post, const float* X, int n, int hw, int C, int groups,
                 const float* save_mean, const float* save_invstd, const float* gamma, float slope,
                 const float* post_out, const float* drop, float* dX, float* dgamma, float* dbeta,
                 const float* post_coef, int post_coef_ld, const int* nvalid, void* workspace, int64_t ws_bytes,
                 void* stream);
/* dX = dY * LeakyReLU'(post) * drop[n][C] (Dropout2d + LeakyReLU backward; post / drop may be
 * null), or with tanh_y != 0: dX = dY * (1 - post^2) (Tanh backward, post = the Tanh output). */
int cgl_act_drop_bwd(const float* dY, const float* post, const float* drop, int n, int hw, int C, float slope,
                     int tanh_y, float* dX, void* stream);
/* cgl_act_drop_bwd for a one-channel map (C == 1, n hw <= 2^21) that also writes the column-sum partials of dX
 * per 256-row chunk, part[(n hw + 255) / 256][2] -- bitwise the chunks the bias-gradient column sum of
 * cgl_conv3x3_bwd_weight computes from dX (G Conv2d(64, 1)'s bias, model/lsgan.py:19-20) -- and
 * cgl_colsum_finalize sums them in chunk order into out[C] (that column sum's finalize). */
int cgl_act_drop_bwd_colsum(const float* dY, const float* post, const float* drop, int n, int hw, int C, float slope,
                            int tanh_y, float* dX, double* part, void* stream);
int cgl_colsum_finalize(const double* part, int nch, int C, float* out, void* stream);
/* nn.Dropout2d(p) scales per (image, channel): 1/(1-p) with probability 1-p, else 0
 * (Philox4x32-10, counter-based: (seed, counter) selects the stream). */
int cgl_dropout2d_mask(float* mask, int n, int C, double p, unsigned long long seed, unsigned long long counter,
                       void* stream);
/* nm (<= 16) masks in one launch: mask j = cgl_dropout2d_mask(masks[j], n[j], C[j], p, seed, counters[j]) */
int cgl_dropout2d_masks(int nm, float* const* masks, const int* n, const int* C, double p, unsigned long long seed,
                        const unsigned long long* counters, void* stream);
/* Layout changes of model/lsgan.py:25 (view(B,128,8,8) of the Linear output) and :96 (view(B,-1)). */
int cgl_nchw_to_nhwc(const float* X, float* Y, int n, int c, int hw, void* stream);
int cgl_nhwc_to_nchw(const float* X, float* Y, int n, int c, int hw, void* stream);
/* Input gradient of the discriminator head Linear(c * hw, 1) (model/lsgan.py:96-97, adv_layer over
 * out.view(B, -1)) written in the NHWC layout of the [n, hw, c] map: dX[m][s][c] = dY[m] * W[c * hw + s]
 * (replaces cgl_dense_bwd_data(K = 1) + cgl_nchw_to_nhwc). c % 4 == 0. */
int cgl_dense1_bwd_data_nhwc(const float* dY, const float* W, float* dX, int n, int c, int hw, void* stream);
/* Forward of the same head from the NHWC map: Y[m] = b + sum_k flat[m][k] W[k], flat[m][c * hw + s] =
 * X[m][s][c], bitwise what cgl_nhwc_to_nchw + cgl_dense_fwd(N = 1) give; flat (may be null) receives the
 * NCHW view (model/lsgan.py:96 out.view(B, -1)). b may be null. c * hw % 256 == 0, <= 1024. */
int cgl_dense1_fwd_nhwc(const float* X, const float* W, const float* b, float* Y, float* flat, int n, int c, int hw,
                        void* stream);
/* The discriminator head of model/lsgan.py (out.view(B, -1) -> adv_layer, :96-97) with its adversarial loss and
 * its input gradient in ONE launch: Y = cgl_dense1_fwd_nhwc (flat as there), per call the mean loss and
 * dY = weight * its gradient as cgl_adv_loss gives them (loss 1 / 2 / 3; one logit), dX = cgl_dense1_bwd_data_nhwc
 * of dY -- bitwise what the three (or, with two calls, four) separate launches produce.  Call 0 is rows [0, n0)
 * (target0, weight0, loss_out0, nvalid0: a short first call as cgl_adv_loss), call 1 rows [n0, n) when n0 < n
 * (the D step's real and fake halves, capgan.py:332-340).  scratch: >= n + 16 floats, zeroed ONCE before the first
 * use (its first word is a monotonic ticket; the last workgroup reduces the losses).  in_coef (may be null): X is
 * the PRE-BatchNorm map and its BatchNorm2d (act none) is applied to every loaded value, scale in_coef[g c + ch],
 * shift in_coef[in_groups c + g c + ch] for rows of group g = row / (n / in_groups) (cgl_bn2d_fwd_stats_coef's
 * coef; bitwise its applied map, which flat receives).  c % 4 == 0, c * hw % 256 == 0, <= 1024. */
int cgl_dense1_head_nhwc(const float* X, const float* W, const float* b, float* Y, float* flat, float* dY, float* dX,
                         int n, int c, int hw, int loss, int n0, int target0, double weight0, float* loss_out0,
                         const int* nvalid0, int target1, double weight1, float* loss_out1, const float* in_coef,
                         int in_groups, float* scratch, void* stream);
/* Mean adversarial loss of one forward call and weight * its gradient (grad may be null):
 * loss 0 CrossEntropy on 2 logits (capgan.py:311), 1 BCELoss on probabilities
 * (CGLGAN/2DMG/main.py:336), 2 MSELoss (LSGAN objective of model/lsgan.py's D), 3 Sigmoid + BCELoss
 * on logits.  target 0 (fake) or 1 (valid); loss_out: device scalar. */
int cgl_adv_loss(const float* x, int M, int C, int loss, int target, double weight, float* loss_out, float* grad,
                 const int* nvalid, void* stream);
/* Exchange weighting: alpha = weights(weighting, lambda, beta, losses[n]) (CGL_WEIGHT_*, the
 * reference's Server.train formulas), then x[0:nx] *= alpha[rank] in place (this worker's
 * contribution before the all-reduce(sum)); alpha_out[n] (device, may be null) receives every alpha.
 * beta_host: host array of n data-size weights (capgan.py:149-153). */
int cgl_weights_scale(int weighting, int n, int rank, float lam, const float* beta_host, const float* losses,
                      float* x, int64_t nx, float* alpha_out, void* stream);
/* dst[r] = src[idx ? idx[r] : row0 + r] for r < nrows (rows of row_floats floats; idx: device int32):
 * the worker's real-batch sampler over a device-resident shard (capgan.py:282,326-332). */
int cgl_gather_rows(const float* src, const int* idx, int64_t row0, int nrows, int row_floats, float* dst,
                    void* stream);
/* optim.Adam step `step` over nt (<= 32) tensors (torch _single_tensor_adam op order), host pointer
 * arrays; no host synchronisation. */
int cgl_adam_multi(int nt, float* const* p, const float* const* g, float* const* m, float* const* v,
                   const int64_t* n, int step, double lr, double beta1, double beta2, double eps, void* stream);

/* ---- device-side round state (graph-replayable fused conv round) ----------------------------
 * The per-round values the ops above take from the host -- the z stream's round (capgan.py:216,219),
 * the Dropout2d counters (model/lsgan.py:78), the Adam step (capgan.py:158,312), the sampler position
 * (capgan.py:282,326-332) -- read from device int32 counters instead, so that one captured round
 * replays as a hipGraph; cgl_counters_add advances them at the end of the round. */
/* cgl_normal_fill with round = *round_dev */
int cgl_normal_fill_dev(float* out, int64_t n, unsigned long long seed, const int* round_dev, int stream_id,
                        void* stream);
/* cgl_dropout2d_masks with counter j = counters[j] + round_stride * (*round_dev) */
int cgl_dropout2d_masks_dev(int nm, float* const* masks, const int* n, const int* C, double p,
                            unsigned long long seed, const unsigned long long* counters, const int* round_dev,
                            unsigned long long round_stride, void* stream);
/* cgl_adam_multi with step = *step_dev + 1 (bias corrections computed on the device) */
int cgl_adam_multi_dev(int nt, float* const* p, const float* const* g, float* const* m, float* const* v,
                       const int64_t* n, const int* step_dev, double lr, double beta1, double beta2, double eps,
                       void* stream);
/* The real batch of round *round_dev, DataLoader(shuffle=True) over the n_src resident rows
 * (capgan.py:282,326-331): each pass is a keyed Feistel permutation of [0, n_src) cut into
 * ceil(n_src / nrows) batches, the last one short; *nv_out receives the batch's real rows (rows past
 * them copy a valid dummy row).  nv_out null: drop_last (whole batches only: pos = round * nrows + r,
 * data epoch pos / per, per = whole batches per pass).  Rows of row_floats (% 4 == 0) floats, 16-byte aligned. */
int cgl_sample_rows_dev(const float* src, int n_src, int nrows, int row_floats, unsigned long long seed,
                        const int* round_dev, float* dst, int* nv_out, void* stream);
/* p[i] += v for i < n (<= 64): advances the device round state */
int cgl_counters_add(int* p, int n, int v, void* stream);

/* ---- evaluation ------------------------------------------------------------------------------
 * KL score of generated 2-D samples (CGLGAN/2DMG/main.py:63-101 plot_2d): np.histogram2d of the
 * real points (rows r * real_stride of real [., 2]) and of the generated points over
 * bins x bins bins of [lo0, hi0] x [lo1, hi1]; counts[2][bins][bins] (real, generated; device int32,
 * may be null) and kl[0] (device double, may be null) = scipy.stats.entropy(gen, real) over the bins
 * whose real count is non-zero.  bins <= 32; one workgroup, stream-ordered. */
int cgl_kl_score(const float* real, int64_t nr, int64_t real_stride, const float* gen, int64_t ng, int64_t gen_stride,
                 int bins, double lo0, double hi0, double lo1, double hi1, int* counts, double* kl, void* stream);

/* Library identification: "<version> gfx950" */
const char* cgl_version(void);

#ifdef __cplusplus
}
#endif
#endif /* CGLGAN_H */
