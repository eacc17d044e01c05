// Do independent branches of a captured hipGraph overlap on the device?  (Decides whether the MLP round
// can hide launch floors by moving off-critical-path launches -- weight gradients, per-layer Adam -- to a
// second captured stream.)  Each kernel: G workgroups, each reads 4 KB its chain's previous kernel wrote
// and writes 4 KB.
//   one   : 2P dependent kernels on one stream (graph)
//   fork  : two independent chains of P kernels captured from two streams (event fork / join, graph)
//   fork2e: the same two chains launched eagerly on two streams (no graph)
//   hipcc --offload-arch=gfx950 -O3 tools/fork_probe.hip -o tools/fork_probe && tools/fork_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_step(const float* in, float* out, int G, int work) {
  const int b = blockIdx.x, t = threadIdx.x;
  const int src = (b * 37 + 11) % G;
  f32x4 v = *(const f32x4*)(in + src * 1024 + t * 4);
  for (int i = 0; i < work; ++i) v = v * 0.999f + 0.001f;   // a little ALU time per kernel
  *(f32x4*)(out + b * 1024 + t * 4) = v;
}

int main() {
  const int P = 10, reps = 200;
  float* buf;
  CK(hipMalloc(&buf, 4 * 1024 * 4096));
  CK(hipMemset(buf, 0, 4 * 1024 * 4096));
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t fork, join, e0, e1;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int G : {64, 256, 1024}) {
    for (int work : {0, 2000}) {
      float* a[2] = {buf, buf + 1024 * 1024};
      float* b[2] = {buf + 2 * 1024 * 1024, buf + 3 * 1024 * 1024};
      auto chain = [&](hipStream_t s, float** x, int n) {
        for (int p = 0; p < n; ++p) k_step<<<G, 256, 0, s>>>(x[p & 1], x[(p + 1) & 1], G, work);
      };
      auto two = [&]() {
        CK(hipEventRecord(fork, s0));
        CK(hipStreamWaitEvent(s1, fork, 0));
        chain(s0, a, P);
        chain(s1, b, P);
        CK(hipEventRecord(join, s1));
        CK(hipStreamWaitEvent(s0, join, 0));
      };
      for (int form = 0; form < 3; ++form) {
        hipGraphExec_t ge = nullptr;
        if (form < 2) {
          hipGraph_t g;
          CK(hipStreamBeginCapture(s0, hipStreamCaptureModeGlobal));
          if (form == 0) chain(s0, a, 2 * P); else two();
          CK(hipStreamEndCapture(s0, &g));
          CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        }
        auto go = [&]() {
          if (ge) CK(hipGraphLaunch(ge, s0)); else two();
        };
        for (int w = 0; w < 10; ++w) go();
        CK(hipStreamSynchronize(s0));
        CK(hipEventRecord(e0, s0));
        for (int r = 0; r < reps; ++r) go();
        CK(hipEventRecord(e1, s0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const char* nm[] = {"one   ", "fork  ", "fork2e"};
        printf("G=%4d work=%4d %s %7.2f us per replay of %d kernels (%.2f us per kernel)\n", G, work, nm[form],
               ms * 1e3 / reps, 2 * P, ms * 1e3 / reps / (2 * P));
      }
    }
  }
  return 0;
}
