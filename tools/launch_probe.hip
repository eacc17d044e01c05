// Where the fixed cost of a dependent kernel launch goes (round 5; tuning aid for the MLP round).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/launch_probe.hip -o tools/launch_probe && tools/launch_probe
// A hipGraph of 28 dependent kernels of 256 workgroups (the round's shape), replayed 200 times; every kernel
// reads what the previous one wrote.  Workgroup 0..255 thread 0 of each kernel stamps the 100 MHz wall clock:
//   e0 entry, e1 after the first kernarg-derived value is in a register, e2 after one dependent scalar load of a
//   descriptor in device memory, e3 after the first vector load of the previous kernel's output, e4 exit.
// Forms: plain; "pad N" = the same with N bytes of straight-line code (s_nop) executed between e3 and e4, to
// price cold instruction fetch per byte of executed code (an s_nop issues in one cycle: 4 KB = 1024 cycles = 0.43 us
// at 2.4 GHz when the fetch keeps up).  Reported: medians over workgroups and replays of
// each interval, and the exit(k) -> entry(k+1) gap (last workgroup out -> first workgroup in).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                      \
      exit(1);                                                                               \
    }                                                                                        \
  } while (0)

struct Desc {
  const float* in;
  float* out;
  int n;
  int pad[13];
};

constexpr int kK = 28, kWG = 256, kW = 5;

template <int PAD>
__global__ __launch_bounds__(256) void k_probe(const Desc* dd, unsigned long long* stamps) {
  const unsigned long long e0 = wall_clock64();
  const int tid = threadIdx.x, b = blockIdx.x;
  unsigned long long* st = stamps + (long)b * kW;
  // e1: a kernarg value in hand (stamps, dd are kernargs: use one through a register dependency)
  const unsigned long long e1 = wall_clock64() + ((unsigned long long)(uintptr_t)dd & 0);
  asm volatile("" ::"s"(dd), "s"(stamps));
  // e2: one dependent scalar load of the descriptor in device memory
  const Desc* __restrict__ d = dd;
  const float* in = d->in;
  float* out = d->out;
  const int n = d->n;
  asm volatile("" ::"s"(in), "s"(out), "s"(n));
  const unsigned long long e2 = wall_clock64();
  // e3: the first vector load of the previous kernel's output
  const int i = (b * 256 + tid) % n;
  float x = in[i];
  asm volatile("" ::"v"(x));
  const unsigned long long e3 = wall_clock64();
  if constexpr (PAD > 0) asm volatile(".rept %0\n s_nop 0\n .endr" ::"i"(PAD / 4));   // PAD bytes of code
  out[i] = x + 1.f;
  if (tid == 0) {
    st[0] = e0;
    st[1] = e1;
    st[2] = e2;
    st[3] = e3;
    st[4] = wall_clock64();
  }
}

template <int PAD>
void run(const char* name, float* bufs[2], Desc* descs, unsigned long long* stamps) {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int k = 0; k < kK; ++k)
    hipLaunchKernelGGL(k_probe<PAD>, dim3(kWG), dim3(256), 0, s, descs + (k & 1), stamps + (long)k * kWG * kW);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int r = 0; r < 20; ++r) CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  std::vector<double> iv[kW - 1], gap;
  std::vector<unsigned long long> h((long)kK * kWG * kW);
  hipEvent_t a, z;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&z));
  double tot = 0;
  const int reps = 50;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(a, s));
    CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(z, s));
    CK(hipStreamSynchronize(s));
    float ms;
    CK(hipEventElapsedTime(&ms, a, z));
    tot += ms;
    CK(hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost));
    for (int k = 0; k < kK; ++k) {
      unsigned long long first = ~0ull, last = 0;
      for (int w = 0; w < kWG; ++w) {
        const unsigned long long* t = &h[((long)k * kWG + w) * kW];
        for (int j = 0; j < kW - 1; ++j) iv[j].push_back((t[j + 1] - t[j]) / 100.0);
        first = std::min(first, t[0]);
        last = std::max(last, t[4]);
      }
      if (k > 0) {
        unsigned long long prev_last = 0;
        for (int w = 0; w < kWG; ++w) prev_last = std::max(prev_last, h[((long)(k - 1) * kWG + w) * kW + 4]);
        gap.push_back(((double)first - (double)prev_last) / 100.0);
      }
    }
  }
  auto med = [](std::vector<double>& v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  printf("%-14s %6.2f us/kernel | entry->kernarg %5.2f  ->desc load %5.2f  ->first vload %5.2f  ->exit %5.2f | gap %5.2f\n",
         name, tot * 1e3 / reps / kK, med(iv[0]), med(iv[1]), med(iv[2]), med(iv[3]), med(gap));
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipStreamDestroy(s));
}

int main() {
  float* bufs[2];
  const int n = kWG * 256;
  for (auto& b : bufs) {
    CK(hipMalloc(&b, n * 4));
    CK(hipMemset(b, 0, n * 4));
  }
  Desc hd[2] = {};
  hd[0].in = bufs[0];
  hd[0].out = bufs[1];
  hd[0].n = n;
  hd[1].in = bufs[1];
  hd[1].out = bufs[0];
  hd[1].n = n;
  Desc* dd;
  CK(hipMalloc(&dd, sizeof(hd)));
  CK(hipMemcpy(dd, hd, sizeof(hd), hipMemcpyHostToDevice));
  unsigned long long* stamps;
  CK(hipMalloc(&stamps, (long)kK * kWG * kW * 8));
  run<0>("plain", bufs, dd, stamps);
  run<4096>("pad 4 KB", bufs, dd, stamps);
  run<16384>("pad 16 KB", bufs, dd, stamps);
  run<65536>("pad 64 KB", bufs, dd, stamps);
  return 0;
}
