// Price of an in-launch grid-wide seam against a kernel boundary on this box (the decision behind a
// persistent MLP round).  P phases; in every phase each 256-thread workgroup reads the
// 4 KB another workgroup wrote in the previous phase and writes 4 KB of its own:
//   chain   P dependent launches captured in one hipGraph (what the round does today)
//   nosync  one launch, the phases back to back with no seam (wrong results; the no-seam floor)
//   fence   one launch, flat seam: payload plain, lane-0 release fence, one agent-scope counter, sc1 poll,
//           acquire fence (the textbook grid barrier)
//   xcd     one launch, XCD-sharded seam: payload plain + release / acquire fences, 8 per-XCD counters, the
//           last arriver of an XCD adds to the top counter, every workgroup polls the top counter
//   wt      one launch, XCD-sharded seam with write-through payload: 16-byte sc1 stores + vmcnt(0) drain,
//           sc1 loads, no fences
// Every poll gives up after a bounded number of tries and raises an error word (no hang on a bad grid).
//   hipcc --offload-arch=gfx950 -O3 tools/barrier_probe.hip -o tools/barrier_probe && tools/barrier_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
#define RLX __ATOMIC_RELAXED
#define AGENT __HIP_MEMORY_SCOPE_AGENT

struct Sync {
  unsigned int* top;     // [32] (one line)
  unsigned int* xc;      // [8][32]
  unsigned int* err;
};

__device__ __forceinline__ bool poll_ge(unsigned int* p, unsigned int target, unsigned int* err) {
  for (int it = 0; it < (1 << 18); ++it) {
    if (__hip_atomic_load(p, RLX, AGENT) - target < 0x80000000u) return true;
    if ((it & 255) == 255 && __hip_atomic_load(err, RLX, AGENT)) return false;   // another poll gave up
    __builtin_amdgcn_s_sleep(1);
  }
  atomicOr(err, 1u);
  return false;
}

template <int MODE>
__device__ __forceinline__ void seam(const Sync& s, unsigned int gen, int G) {
  // gen: 1-based count of seams passed by this launch sequence (monotonic across launches)
  __syncthreads();
  if (threadIdx.x == 0) {
    if (MODE != 3) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (MODE == 1) {
      __hip_atomic_fetch_add(s.top, 1u, RLX, AGENT);
      poll_ge(s.top, gen * (unsigned)G, s.err);
    } else {
      const int x = blockIdx.x & 7;
      const unsigned per = (unsigned)(G / 8);
      const unsigned old = __hip_atomic_fetch_add(s.xc + x * 32, 1u, RLX, AGENT);
      if (old + 1 == gen * per) __hip_atomic_fetch_add(s.top, 1u, RLX, AGENT);
      poll_ge(s.top, gen * 8u, s.err);
    }
    if (MODE != 3) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// MODE 0 nosync, 1 fence, 2 xcd, 3 wt (write-through); CHAIN: one phase per launch
template <int MODE>
__global__ __launch_bounds__(256) void k_phases(float* buf, int G, int P, int ph0, unsigned int gen0, Sync s,
                                                float* sink) {
  const int b = blockIdx.x, t = threadIdx.x;
  const int src = (b * 37 + 11) % G;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  auto rs = __builtin_amdgcn_make_buffer_rsrc(buf, (short)0, 2 * G * 4096, 0x00020000);
  for (int p = 0; p < P; ++p) {
    const int ph = ph0 + p;
    const float* in = buf + (long)((ph + 1) & 1) * G * 1024;
    float* out = buf + (long)(ph & 1) * G * 1024;
    f32x4 v;
    if (MODE == 3) {
      const int off = (int)((((ph + 1) & 1) * G * 1024 + src * 1024 + t * 4) * 4);
      v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16));
    } else {
      v = *(const f32x4*)(in + src * 1024 + t * 4);
    }
    acc += v;
    const f32x4 w = v * 0.5f + 1.f;
    if (MODE == 3) {
      const int off = (int)(((ph & 1) * G * 1024 + b * 1024 + t * 4) * 4);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, w), rs, off, 0, 16);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      *(f32x4*)(out + b * 1024 + t * 4) = w;
    }
    if (MODE != 0 && p + 1 < P) seam<MODE>(s, gen0 + p + 1, G);
  }
  if (acc[0] == 1234.5f) sink[0] = acc[1];
}

int main() {
  const int P = 28, reps = 100;
  float *buf, *sink;
  unsigned int* words;
  CK(hipMalloc(&buf, 2 * 1024 * 4096));
  CK(hipMalloc(&sink, 64));
  CK(hipMalloc(&words, 4096 * 4));
  CK(hipMemset(buf, 0, 2 * 1024 * 4096));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int dev = 0;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, dev));
  printf("device %s, %d CUs; %d phases of 4 KB read + 4 KB write per workgroup\n", prop.name,
         prop.multiProcessorCount, P);
  for (int G : {256, 512, 1024}) {
    Sync s;
    CK(hipMemset(words, 0, 4096 * 4));
    s.top = words;
    s.xc = words + 64;
    s.err = words + 1024;
    // chain of launches (hipGraph)
    {
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
      for (int p = 0; p < P; ++p) k_phases<0><<<G, 256, 0, st>>>(buf, G, 1, p, 0, s, sink);
      CK(hipStreamEndCapture(st, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      for (int w = 0; w < 10; ++w) CK(hipGraphLaunch(ge, st));
      CK(hipEventRecord(e0, st));
      for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, st));
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("G=%4d chain   %7.2f us per phase (%.1f us per %d-launch graph)\n", G, ms * 1e3 / reps / P, ms * 1e3 / reps, P);
    }
    for (int mode = 0; mode < 4; ++mode) {
      CK(hipMemset(words, 0, 4096 * 4));
      unsigned int gen = 0;
      auto launch = [&]() {
        if (mode == 0) k_phases<0><<<G, 256, 0, st>>>(buf, G, P, 0, gen, s, sink);
        if (mode == 1) k_phases<1><<<G, 256, 0, st>>>(buf, G, P, 0, gen, s, sink);
        if (mode == 2) k_phases<2><<<G, 256, 0, st>>>(buf, G, P, 0, gen, s, sink);
        if (mode == 3) k_phases<3><<<G, 256, 0, st>>>(buf, G, P, 0, gen, s, sink);
        gen += P - 1;
      };
      for (int w = 0; w < 10; ++w) launch();
      CK(hipStreamSynchronize(st));
      CK(hipEventRecord(e0, st));
      for (int r = 0; r < reps; ++r) launch();
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      unsigned int err = 0;
      CK(hipMemcpy(&err, s.err, 4, hipMemcpyDeviceToHost));
      const char* nm[] = {"nosync", "fence ", "xcd   ", "wt    "};
      printf("G=%4d %s %7.2f us per phase (%.1f us per launch)%s\n", G, nm[mode], ms * 1e3 / reps / P, ms * 1e3 / reps,
             err ? "  [poll gave up]" : "");
    }
  }
  return 0;
}
