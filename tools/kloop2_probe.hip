// k-loop probe, round 6: operand DELIVERY of the MLP forward GEMM (fragment-packed A and B, 1x1 32x32 block per
// wave, the round's G3 / G4 forward geometry WM = 2, WN = 1, WK = 2: a 256-thread workgroup owns a 64 x 32 tile, the
// two waves of a k-half share the B chunk).  Variants, all with the same MFMA sequence (two alternating accumulation
// chains, chunk order, fixed-order in-workgroup k reduction), so every variant must give bitwise the same C:
//   R<S>  register rotation of S chunk sets (cgl_gemm_f32's loop: 16-byte loads straight into fragment registers)
//   L<D>  LDS ring of D chunks filled by global_load_lds_dwordx4: A private per wave, B SHARED by the two waves of
//         a k-half (each loads one 1 KB half), one raw s_barrier per chunk, counted vmcnt
//   Q<D>  the same ring with B private (no sharing, no barrier): the ring depth alone
// Each timed twice: warm (200 back-to-back launches) and as in the round (a scrub kernel before every launch rewrites
// A from every CU and streams 48 MB through the L2s, so A comes back from the Infinity Cache as a freshly written
// producer output does; only the GEMM launch is inside the events).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/kloop2_probe.hip -o tools/kloop2_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(1))) const f32x4* gcf4p;
typedef __attribute__((address_space(1))) const void* gvp;
typedef __attribute__((address_space(3))) void* lvp;

struct P { const float* A; const float* B; float* C; int M, N, K, tiles_m, tiles_n; };

__device__ __forceinline__ void glds(const float* g, float* l) {
  __builtin_amdgcn_global_load_lds((gvp)g, (lvp)l, 16, 0, 0);
}

// L2 prefetch workgroups (blockIdx >= the tile count): the workgroup assumes the round-robin XCD placement of
// blocks (b % 8; a speed assumption only, never a correctness one), finds the tile range the XCD-contiguous order
// gives that XCD, and pulls the A row blocks and B column blocks of those tiles into the XCD's L2 in the order the
// two k-halves consume them (chunk cb + i and ch + i alternately), 1 KB per global_load_lds_dwordx4 into a scratch
// LDS slot it never reads.  pf = prefetch workgroups per XCD.
__device__ void prefetch_wg(const P& p, int pf, float* lds) {
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int nwg = p.tiles_m * p.tiles_n;
  const int b = blockIdx.x - nwg;
  const int xcd = b & 7, j = b >> 3;                 // j-th prefetcher of this XCD
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int u0 = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
  const int u1 = u0 + q8 + (xcd < r8 ? 1 : 0);
  if (u1 <= u0) return;
  const int tn0 = u0 / p.tiles_m, tn1 = (u1 - 1) / p.tiles_m;
  const int tm0 = (tn0 == tn1) ? u0 % p.tiles_m : 0, tm1 = (tn0 == tn1) ? (u1 - 1) % p.tiles_m : p.tiles_m - 1;
  const int na = (tm1 - tm0 + 1) * 2, nb = tn1 - tn0 + 1;        // A 32-row blocks, B 32-column blocks
  const int nch = p.K / 16, ch = nch / 2;
  const int per = na + nb;                                         // 2 KB pieces per chunk
  const long total = (long)nch * per * 2;                          // 1 KB halves
  float* slot = lds + wave * 256;
  int inflight = 0;
  for (long h = (long)j * 4 + wave; h < total; h += (long)pf * 4) {
    const long piece = h >> 1;
    const int half = (int)(h & 1);
    const int ci = (int)(piece / per), k = (int)(piece % per);
    const int c = (ci & 1) ? ch + (ci >> 1) : (ci >> 1);          // the two k-halves' chunks interleaved
    if (c >= nch) continue;
    const float* src = (k < na) ? p.A + ((long)(tm0 * 2 + k) * nch + c) * 512 : p.B + ((long)(tn0 + k - na) * nch + c) * 512;
    __builtin_amdgcn_global_load_lds((gvp)(src + half * 256 + lane * 4), (lvp)slot, 16, 0, 0);
    if (++inflight == 48) {
      asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
      inflight = 24;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int V, int D, int PF = 0>
__global__ __launch_bounds__(256) void kp(P p) {
  extern __shared__ float lds[];
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int wm = wave >> 1, wk = wave & 1;
  if (PF > 0 && (int)blockIdx.x >= p.tiles_m * p.tiles_n) {
    prefetch_wg(p, PF, lds);
    return;
  }
  // XCD-contiguous n-major tile order (as cgl_gemm_f32)
  const int nwg = p.tiles_m * p.tiles_n, local = blockIdx.x;
  const int xcd = local & 7, pos = local >> 3, q8 = nwg >> 3, r8 = nwg & 7;
  const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + pos;
  const int tn = tile / p.tiles_m, tm = tile % p.tiles_m;
  const int nch = p.K / 16;
  const int cb = wk * nch / 2, ce = (wk + 1) * nch / 2;
  const float* Ab = p.A + (long)(tm * 2 + wm) * nch * 512 + lane * 4;   // this wave's A block, lane's float4
  const float* Bb = p.B + (long)tn * nch * 512 + lane * 4;
  f32x16 acc0 = {}, acc1 = {};
  auto mm = [&](const float (&a)[8], const float (&b)[8]) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      if (q & 1) acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q], b[q], acc1, 0, 0, 0);
      else acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q], b[q], acc0, 0, 0, 0);
    }
  };
  if constexpr (V == 0 || V == 3) {
    // V == 3: every workgroup walks its k-range from a rotated start (spread evenly over the XCD's workgroups), so
    // the XCD's workgroups first touch different chunks at the same time instead of all waiting on the same lines
    constexpr int S = D;
    const int nk = ce - cb;
    const int upx = q8 + (xcd < r8 ? 1 : 0);
    const int rot = (V == 3 && upx > 0) ? (int)(((long)pos * nk) / upx) : 0;
    auto cmap = [&](int c) { int i = c - cb + rot; if (i >= nk) i -= nk; return cb + i; };
    auto ld = [&](int c0, float (&a)[8], float (&b)[8]) {
      const int c = cmap(c0);
      const f32x4 x = *(gcf4p)(Ab + c * 512), y = *(gcf4p)(Ab + c * 512 + 256);
      const f32x4 u = *(gcf4p)(Bb + c * 512), v = *(gcf4p)(Bb + c * 512 + 256);
      a[0] = x[0]; a[1] = x[1]; a[2] = x[2]; a[3] = x[3]; a[4] = y[0]; a[5] = y[1]; a[6] = y[2]; a[7] = y[3];
      b[0] = u[0]; b[1] = u[1]; b[2] = u[2]; b[3] = u[3]; b[4] = v[0]; b[5] = v[1]; b[6] = v[2]; b[7] = v[3];
    };
    float a[S][8], b[S][8];
#pragma unroll
    for (int s = 0; s < S; ++s) ld(min(cb + s, ce - 1), a[s], b[s]);
    int c = cb;
    for (; c + S <= ce; c += S) {
#pragma unroll
      for (int s = 0; s < S; ++s) {
        mm(a[s], b[s]);
        __builtin_amdgcn_sched_barrier(0);
        ld(min(c + s + S, ce - 1), a[s], b[s]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int s = 0; s < S - 1; ++s)
      if (c + s < ce) mm(a[s], b[s]);
  } else {
    // ring slot layout per k-half group g = wk: [D][A wm0 512 | A wm1 512 | B 512] floats (V == 1)
    //                                           [D][A wm0 | A wm1 | B wm0 512 | B wm1 512]  (V == 2, B private)
    constexpr int SLOT = (V == 1) ? 1536 : 2048;
    float* ring = lds + wk * D * SLOT;
    constexpr int NL = (V == 1) ? 3 : 4;     // glds per wave per chunk
    auto issue = [&](int cv, int c) {   // chunk c into the slot of virtual chunk cv (cv > c past the end)
      float* sl = ring + (cv % D) * SLOT;
      const float* ga = Ab + (long)c * 512;
      glds(ga, sl + wm * 512);               // (lane-linear: lane l's 16 B at l * 16)
      glds(ga + 256, sl + wm * 512 + 256);
      if (V == 1) {
        glds(Bb + (long)c * 512 + wm * 256, sl + 1024 + wm * 256);
      } else {
        glds(Bb + (long)c * 512, sl + 1024 + wm * 512);
        glds(Bb + (long)c * 512 + 256, sl + 1024 + wm * 512 + 256);
      }
    };
    const int n = ce - cb;
    for (int i = 0; i < D - 1; ++i) issue(cb + i, min(cb + i, ce - 1));
    for (int c = cb; c < ce; ++c) {
      // chunk c's own loads done: D - 2 chunks stay in flight
      if constexpr (NL * (D - 2) == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else if constexpr (NL * (D - 2) == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      else if constexpr (NL * (D - 2) == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if constexpr (NL * (D - 2) == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else if constexpr (NL * (D - 2) == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if constexpr (NL * (D - 2) == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      else if constexpr (NL * (D - 2) == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else if constexpr (NL * (D - 2) == 18) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
      else if constexpr (NL * (D - 2) == 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
      else static_assert(NL * (D - 2) < 0, "add the vmcnt case");
      // the partner's half of B landed; every wave is past its reads of slot (c - 1) % D
      if (V == 1) __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      // (past the end: the last chunk again, into the free slot, so the counted waits stay exact)
      issue(c + D - 1, min(c + D - 1, ce - 1));
      const float* sl = ring + (c % D) * SLOT;
      const f32x4 x = *(const f32x4*)(sl + wm * 512 + lane * 4), y = *(const f32x4*)(sl + wm * 512 + 256 + lane * 4);
      const float* bs = sl + 1024 + (V == 1 ? 0 : wm * 512);
      const f32x4 u = *(const f32x4*)(bs + lane * 4), v = *(const f32x4*)(bs + 256 + lane * 4);
      const float a[8] = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
      const float b[8] = {u[0], u[1], u[2], u[3], v[0], v[1], v[2], v[3]};
      mm(a, b);
    }
    (void)n;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) acc0[r] += acc1[r];
  // fixed-order k reduction (wk = 1 into wk = 0) through LDS
  __syncthreads();
  float* red = lds;
  if (wk == 1)
    for (int r = 0; r < 16; ++r) red[(wm * 16 + r) * 64 + lane] = acc0[r];
  __syncthreads();
  if (wk == 1) return;
  for (int r = 0; r < 16; ++r) acc0[r] += red[(wm * 16 + r) * 64 + lane];
  float* C = p.C + ((long)tile * 2 + wm) * 1024;
  for (int q = 0; q < 4; ++q) *(f32x4*)(C + q * 256 + lane * 4) = f32x4{acc0[4 * q], acc0[4 * q + 1], acc0[4 * q + 2], acc0[4 * q + 3]};
}

// the round's data state before a forward GEMM: its A operand just written by the producer (every CU), the L2s
// full of other traffic
__global__ void scrub(float* A, long na, const float* junk, long nj, float* sink) {
  const long i0 = (long)blockIdx.x * blockDim.x + threadIdx.x, st = (long)gridDim.x * blockDim.x;
  for (long i = i0; i < na; i += st) A[i] = A[i] * 1.0f + 0.0f;
  float s = 0.f;
  for (long i = i0 * 4; i < nj; i += st * 4) {
    const f32x4 v = *(const f32x4*)(junk + i);
    s += v[0] + v[1] + v[2] + v[3];
  }
  if (s == 12345.f) sink[0] = s;
}

int main() {
  struct Sh { const char* name; int M, N, K; } shapes[] = {
      {"G4 fwd", 512, 800, 1024}, {"G3 fwd", 512, 1024, 512}, {"D0 fwd", 512, 512, 784}, {"G4 dA", 256, 1024, 784},
      {"G3 dA", 256, 512, 1024}};
  const long big = 4l << 20, nj = 12l << 20;
  float *A, *B, *C, *junk, *sink;
  CK(hipMalloc(&A, big * 4)); CK(hipMalloc(&B, big * 4)); CK(hipMalloc(&C, big * 4));
  CK(hipMalloc(&junk, nj * 4)); CK(hipMalloc(&sink, 64));
  std::vector<float> h(big);
  for (long i = 0; i < big; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  CK(hipMemcpy(A, h.data(), big * 4, hipMemcpyHostToDevice));
  for (long i = 0; i < big; ++i) h[i] = (float)((i * 40503u + 7) % 997) / 997.f - 0.5f;
  CK(hipMemcpy(B, h.data(), big * 4, hipMemcpyHostToDevice));
  CK(hipMemset(junk, 0, nj * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  struct Var { const char* name; void (*k)(P); int shmem; int pf; };
  Var vars[] = {{"R3", kp<0, 3>, 8192, 0}, {"R3/Aonly", kp<0, 3>, 8192, -1}, {"R3/junkonly", kp<0, 3>, 8192, -2},
                {"R3/Bonly", kp<0, 3>, 8192, -3}};
  for (auto& v : vars) CK(hipFuncSetAttribute((const void*)v.k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  std::vector<float> ref(big), out(big);
  for (auto& s : shapes) {
    P p{A, B, C, s.M, s.N, s.K, s.M / 64, s.N / 32};
    const int grid0 = p.tiles_m * p.tiles_n;
    const long nc = (long)s.M * s.N;
    printf("%-6s M=%4d N=%4d K=%4d grid %3d |", s.name, s.M, s.N, s.K, grid0);
    for (int vi = 0; vi < (int)(sizeof(vars) / sizeof(vars[0])); ++vi) {
      Var& v = vars[vi];
      const int grid = grid0 + 8 * (v.pf > 0 ? v.pf : 0);
      CK(hipMemset(C, 0, nc * 4));
      hipLaunchKernelGGL(v.k, dim3(grid), dim3(256), v.shmem, 0, p);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(vi == 0 ? ref.data() : out.data(), C, nc * 4, hipMemcpyDeviceToHost));
      const bool same = vi == 0 || std::memcmp(ref.data(), out.data(), nc * 4) == 0;
      const int reps = 200;
      for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(v.k, dim3(grid), dim3(256), v.shmem, 0, p);
      CK(hipEventRecord(e0));
      for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(v.k, dim3(grid), dim3(256), v.shmem, 0, p);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double warm = ms * 1e3 / reps;
      double cold = 0;
      const int creps = 60;
      for (int i = 0; i < creps; ++i) {
        // scrub modes: default both (A rewritten + 48 MB through the L2s); -1 A only; -2 junk only; -3 B only
        if (v.pf == -3)
          hipLaunchKernelGGL(scrub, dim3(1024), dim3(256), 0, 0, const_cast<float*>(p.B), (long)s.N * s.K, junk, 0l, sink);
        else
          hipLaunchKernelGGL(scrub, dim3(1024), dim3(256), 0, 0, A, v.pf == -2 ? 0l : (long)s.M * s.K, junk,
                             v.pf == -1 ? 0l : nj, sink);
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(v.k, dim3(grid), dim3(256), v.shmem, 0, p);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        cold += ms * 1e3;
      }
      cold /= creps;
      printf(" %s %5.2f/%5.2f%s |", v.name, warm, cold, same ? "" : " MISMATCH");
      fflush(stdout);
    }
    printf("\n");
  }
  printf("(us per launch: warm / after a scrub; MISMATCH: C differs bitwise from R3)\n");
  return 0;
}
