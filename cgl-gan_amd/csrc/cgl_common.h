// Device / host helpers shared by the two translation units of libcglgan_hip (the MLP step:
// cgl_runtime.hip with cgl_gemm.hip + cgl_kernels.hip; the conv path: cgl_conv_tu.hip with
// cgl_conv.hip + cgl_eval.hip).  Included by cgl_internal.h.
#pragma once

// Launch batching (cgl_conv_batch_begin / _end, cgl_conv.hip): while the calling thread has a batch open,
// only the batchable entry points may be called (they record instead of launching); every other entry point
// that would launch or synchronise returns CGL_E_STATE instead of running ahead of the deferred launches.
bool cgl_launch_batch_open();
#define CGL_BATCH_GUARD()                             \
  do {                                                \
    if (cgl_launch_batch_open()) return CGL_E_STATE;  \
  } while (0)

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef CGL_GLOBAL unsigned int cgl_gu32;
typedef CGL_GLOBAL unsigned long long cgl_gu64;
__device__ __forceinline__ void cgl_pub2f(float* p, float a, float b) {
  const unsigned long long v = (unsigned long long)__float_as_uint(a) | ((unsigned long long)__float_as_uint(b) << 32);
  __hip_atomic_store((cgl_gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void cgl_pubd(double* p, double a) {
  __hip_atomic_store((cgl_gu64*)p, (unsigned long long)__double_as_longlong(a), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ unsigned long long cgl_ld64(const void* p) {
  return __hip_atomic_load((cgl_gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ float cgl_lerp(float self, float end, float w) {
  // at::lerp: |w| < 0.5 ? self + w * (end - self) : end - (end - self) * (1 - w)
  return fabsf(w) < 0.5f ? self + w * (end - self) : end - (end - self) * (1.f - w);
}

__device__ __forceinline__ float cgl_softmax_at(const float* x, int n, int i) {
  float mx = x[0];
  for (int q = 1; q < n; ++q) mx = fmaxf(mx, x[q]);
  float s = 0.f;
  for (int q = 0; q < n; ++q) s += expf(x[q] - mx);
  return expf(x[i] - mx) / s;
}

// tmp / tmp2: 2 x CGL_MAX_WORKERS floats of caller scratch -- LDS in every kernel that calls this (per-lane
// arrays indexed by a runtime N would put the whole kernel on a private scratch segment)
__device__ inline void cgl_weights(int mode, int N, float lam, const float* beta, const float* loss, float* alpha,
                                   float* tmp, float* tmp2) {
  if (mode == CGL_W_MEAN) {
    for (int i = 0; i < N; ++i) alpha[i] = 1.f / N;
    return;
  }
  if (mode == CGL_W_MIX_SINGLE) {
    for (int i = 0; i < N; ++i) tmp[i] = beta[i] * lam * loss[i];
    for (int i = 0; i < N; ++i) alpha[i] = cgl_softmax_at(tmp, N, i);
    return;
  }
  for (int i = 0; i < N; ++i) tmp[i] = lam * loss[i];
  for (int i = 0; i < N; ++i) tmp2[i] = cgl_softmax_at(tmp, N, i);   // softmax(lambda * l)
  if (mode == CGL_W_CGLGAN) {
    for (int i = 0; i < N; ++i) alpha[i] = (beta[i] + tmp2[i]) * 0.5f;
    return;
  }
  if (mode == CGL_W_CAPGAN) {
    for (int i = 0; i < N; ++i) tmp[i] = tmp2[i] * beta[i];          // softmax(a * beta)
  } else {  // CGL_W_MIX_DOUBLE
    for (int i = 0; i < N; ++i) tmp[i] = beta[i] * tmp2[i];
  }
  for (int i = 0; i < N; ++i) alpha[i] = cgl_softmax_at(tmp, N, i);
}

__device__ __forceinline__ void cgl_philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)M0 * c[0], p1 = (uint64_t)M1 * c[2];
    const uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0;
    const uint32_t h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
    const uint32_t n0 = h1 ^ c[1] ^ k0, n2 = h0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = l1; c[2] = n2; c[3] = l0;
    k0 += W0; k1 += W1;
  }
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// One Adam element update in torch 2.10 _single_tensor_adam's operation order (foreach=False,
// capgan.py:158,312): m = lerp(m, g, 1 - beta1), v = v beta2 + (1 - beta2) g g,
// p += -step_size m / (sqrt(v) / sqrt(bias_correction2) + eps).  Shared by cgl_adam and the Adam
// folded into the GEMM launches (cgl_gemm.hip) so that both round identically.
// torch's _single_tensor_adam step for one element.  The fused multiply-adds are written out and contraction is
// off for the rest, so every kernel that inlines this (cgl_adam, the GEMM-epilogue Adam, the tiled cgl_adam_pack)
// computes bitwise the same value whatever the surrounding code lets the compiler fuse (a vectorised caller had
// been contracted differently).  The FMAs are the ones the compiler chose for the scalar kernel before: exp_avg.lerp_
// (at::lerp's two branches as FMAs), exp_avg_sq.mul_(b2).addcmul_(g, g, 1 - b2) = fma((1 - b2) g, g, v b2).
__device__ __forceinline__ void cgl_adam_update(float& p, float g, float& m, float& v, float ss, float bc, float b2,
                                                float w1, float w2, float eps) {
#pragma clang fp contract(off)
  const float d = g - m;
  m = fabsf(w1) < 0.5f ? fmaf(w1, d, m) : fmaf(-d, 1.f - w1, g);
  v = fmaf(w2 * g, g, v * b2);
  const float denom = sqrtf(v) / bc + eps;
  p = p + (-ss) * m / denom;
}

// outputs 4q .. 4q+3 of the N(0,1) stream (seed, round, stream_id)
__device__ __forceinline__ void cgl_normal_at(long q, float* out, long n, unsigned long long seed, uint32_t round,
                                              int stream_id) {
  if (q * 4 >= n) return;
  uint32_t c[4] = {(uint32_t)q, (uint32_t)(q >> 32), round, (uint32_t)stream_id};
  cgl_philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const float inv = 2.3283064365386963e-10f;   // 2^-32
  float z[4];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const float u1 = ((float)c[2 * j] + 1.0f) * inv;   // (0, 1]
    const float u2 = (float)c[2 * j + 1] * inv;
    const float rr = sqrtf(-2.0f * logf(u1));
    float s, co;
    sincosf(6.283185307179586f * u2, &s, &co);
    z[2 * j] = rr * co;
    z[2 * j + 1] = rr * s;
  }
  for (int j = 0; j < 4; ++j)
    if (q * 4 + j < n) out[q * 4 + j] = z[j];
}

// Shuffle sampler: keyed Feistel permutation of [0, n) per data epoch (cycle walking).
__device__ __forceinline__ uint32_t cgl_hash(uint32_t x, uint32_t k) {
  x ^= k;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

__device__ inline uint32_t cgl_permute(uint32_t i, uint32_t n, uint32_t key) {
  int bits = 2;
  while ((1u << bits) < n) ++bits;
  if (bits & 1) ++bits;
  const int hb = bits / 2;
  const uint32_t mask = (1u << hb) - 1;
  uint32_t x = i;
  do {
    uint32_t l = x >> hb, r = x & mask;
    for (int round = 0; round < 4; ++round) {
      const uint32_t t = l ^ (cgl_hash(r, key + 0x9e3779b9u * (round + 1)) & mask);
      l = r;
      r = t;
    }
    x = (l << hb) | r;
  } while (x >= n);
  return x;
}
