// Per-launch cost of dependent kernels in a replayed hipGraph (tuning aid for the MLP round):
// 28 kernels of 256 workgroups each, every kernel reading what the previous one wrote, in forms that
// differ only in where the kernel's descriptor lives and how many dependent memory round trips it makes.
//   hipcc --offload-arch=gfx950 -O3 tools/latency_probe.hip -o tools/latency_probe && tools/latency_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

struct Desc { float* in; float* out; int n; int pad[13]; };

__global__ void k_empty(float* p) { if (p && threadIdx.x == 9999) p[0] = 1.f; }
// descriptor in device memory: 1 dependent load (desc) then the data load, then store
__global__ void k_desc(const Desc* d) {
  const Desc* __restrict__ dd = d;
  const int i = blockIdx.x * 256 + threadIdx.x;
  float* in = dd->in; float* out = dd->out;
  out[i] = in[i] + 1.f;
}
// descriptor by value (kernarg segment)
__global__ void k_arg(Desc d) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  d.out[i] = d.in[i] + 1.f;
}
// by value + an extra dependent load (partials -> data index)
__global__ void k_arg2(Desc d) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int j = (int)d.in[(i * 7) % d.n];
  d.out[i] = d.in[(i + (j & 1)) % d.n] + 1.f;
}
// by value, no data load: store only
__global__ void k_store(Desc d) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  d.out[i] = 1.f;
}

int main() {
  const int n = 256 * 256, L = 28;
  float *a, *b;
  CK(hipMalloc(&a, n * 4)); CK(hipMalloc(&b, n * 4));
  CK(hipMemset(a, 0, n * 4)); CK(hipMemset(b, 0, n * 4));
  Desc* dd; CK(hipMalloc(&dd, L * sizeof(Desc)));
  Desc hd[L];
  for (int i = 0; i < L; ++i) { hd[i].in = (i & 1) ? b : a; hd[i].out = (i & 1) ? a : b; hd[i].n = n; }
  CK(hipMemcpy(dd, hd, sizeof(hd), hipMemcpyHostToDevice));
  hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const char* names[] = {"empty", "desc-in-memory + data load", "desc-by-value + data load", "by-value + 2 dependent loads",
                         "by-value store only"};
  for (int form = 0; form < 5; ++form) {
    hipGraph_t g; hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < L; ++i) {
      if (form == 0) k_empty<<<256, 256, 0, s>>>(nullptr);
      if (form == 1) k_desc<<<256, 256, 0, s>>>(dd + i);
      if (form == 2) k_arg<<<256, 256, 0, s>>>(hd[i]);
      if (form == 3) k_arg2<<<256, 256, 0, s>>>(hd[i]);
      if (form == 4) k_store<<<256, 256, 0, s>>>(hd[i]);
    }
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int w = 0; w < 20; ++w) CK(hipGraphLaunch(ge, s));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int reps = 200;
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-32s %.2f us per kernel (graph of %d, %.1f us per replay)\n", names[form], ms * 1e3 / reps / L, L, ms * 1e3 / reps);
  }
  return 0;
}
