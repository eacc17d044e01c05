// Evaluation of generated 2-D samples: the KL score of CGLGAN/2DMG/main.py:63-101 (plot_2d).
//
// The reference bins a strided subsample of the real test set and of the servers' generated points
// with np.histogram2d(x, y, bins=16, range=[[-1, 1], [-1, 1]]), keeps the bins whose REAL count is
// non-zero (row-major over the x bin, then the y bin) and scores scipy.stats.entropy(gen, real) =
// sum p log(p / q) over those bins, p = gen / sum(gen), q = real / sum(real).
//
// One workgroup per launch (a few thousand points): counts in LDS with integer atomics (order-free,
// exact), bin index = np.histogramdd's rule -- searchsorted(edges, v, 'right') - 1 over the edges of
// np.linspace(lo, hi, bins + 1) computed with the same double roundings (k * step + lo, last = hi),
// a value equal to the last edge goes to the last bin, values outside [lo, hi] (and NaN) are
// dropped.  The KL sum runs in double in numpy's pairwise-summation order over the kept bins.
#include "cgl_internal.h"

#define CGL_HIST_MAXB 32

__device__ __forceinline__ int cgl_hist_bin(double v, const double* __restrict__ edges, int bins) {
  if (!(v >= edges[0]) || !(v <= edges[bins])) return -1;     // outside the range (or NaN)
  if (v == edges[bins]) return bins - 1;                       // histogramdd's on_edge rule
  int lo = 0, hi = bins;                                       // searchsorted 'right' - 1
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (edges[mid] <= v) lo = mid; else hi = mid;
  }
  return lo;
}

// numpy's pairwise_sum for float64 (n <= 8: sequential from -0.0; <= 128: 8 accumulators; else
// halves rounded down to a multiple of 8), over a[0..n).
__device__ double cgl_np_block_sum(const double* a, int n) {
  if (n < 8) {
    double r = -0.0;
    for (int i = 0; i < n; ++i) r += a[i];
    return r;
  }
  double r[8];
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  int i = 8;
  for (; i < n - (n % 8); i += 8)
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += a[i];
  return res;
}
__device__ double cgl_np_pairwise_sum(const double* a, int n) {
  // explicit post-order walk of numpy's split tree (no recursion): n <= CGL_HIST_MAXB^2 = 1024
  // needs 4 levels; (left + right) combined exactly as numpy does
  int st_off[16], st_n[16], state[16], sp = 0;
  double vals[16];
  int vsp = 0;
  st_off[0] = 0; st_n[0] = n; state[0] = 0; sp = 1;
  while (sp > 0) {
    const int top = sp - 1;
    const int off = st_off[top], cnt = st_n[top];
    if (cnt <= 128) {
      vals[vsp++] = cgl_np_block_sum(a + off, cnt);
      --sp;
      continue;
    }
    int n2 = cnt / 2;
    n2 -= n2 % 8;
    if (state[top] == 0) {            // push left
      state[top] = 1;
      st_off[sp] = off; st_n[sp] = n2; state[sp] = 0; ++sp;
    } else if (state[top] == 1) {     // push right
      state[top] = 2;
      st_off[sp] = off + n2; st_n[sp] = cnt - n2; state[sp] = 0; ++sp;
    } else {                          // combine
      const double r = vals[--vsp], l = vals[--vsp];
      vals[vsp++] = l + r;
      --sp;
    }
  }
  return vals[0];
}

struct CglKlArgs {
  const float* real; long nr; long sr;    // rows [nr] of 2 floats, stride sr rows (the strided subsample)
  const float* gen; long ng; long sg;
  int bins;
  double lo0, hi0, lo1, hi1;
  int* counts;                            // [2][bins][bins] (real, gen), may be null
  double* kl;                             // [1], may be null
};

__global__ __launch_bounds__(1024) void cgl_hist2d_kl_k(CglKlArgs a) {
  __shared__ int h[2][CGL_HIST_MAXB * CGL_HIST_MAXB];
  __shared__ double e0[CGL_HIST_MAXB + 1], e1[CGL_HIST_MAXB + 1];
  __shared__ double pk[CGL_HIST_MAXB * CGL_HIST_MAXB], qk[CGL_HIST_MAXB * CGL_HIST_MAXB];
  __shared__ int nkeep;
  const int B = a.bins, BB = B * B;
  for (int i = threadIdx.x; i < 2 * CGL_HIST_MAXB * CGL_HIST_MAXB; i += blockDim.x) (&h[0][0])[i] = 0;
  if (threadIdx.x <= B) {
    // np.linspace(lo, hi, B + 1): step = (hi - lo) / B; y = k * step + lo; y[-1] = hi
    const int k = threadIdx.x;
    const double s0 = (a.hi0 - a.lo0) / B, s1 = (a.hi1 - a.lo1) / B;
    e0[k] = k == B ? a.hi0 : __dadd_rn(__dmul_rn((double)k, s0), a.lo0);
    e1[k] = k == B ? a.hi1 : __dadd_rn(__dmul_rn((double)k, s1), a.lo1);
  }
  __syncthreads();
  for (long i = threadIdx.x; i < a.nr + a.ng; i += blockDim.x) {
    const bool g = i >= a.nr;
    const float* p = g ? a.gen + (i - a.nr) * a.sg * 2 : a.real + i * a.sr * 2;
    const int bx = cgl_hist_bin((double)gld(p), e0, B), by = cgl_hist_bin((double)gld(p + 1), e1, B);
    if (bx >= 0 && by >= 0) atomicAdd(&h[g ? 1 : 0][bx * B + by], 1);
  }
  __syncthreads();
  if (a.counts)
    for (int i = threadIdx.x; i < 2 * BB; i += blockDim.x) a.counts[i] = h[i / BB][i % BB];
  if (!a.kl) return;
  if (threadIdx.x == 0) {
    // kept bins in row-major order (main.py:87-91), then entropy(g, r) (scipy: normalise both by
    // np.sum, sum of rel_entr(p, q))
    int n = 0;
    for (int i = 0; i < BB; ++i)
      if (h[0][i] != 0) {
        qk[n] = (double)h[0][i];
        pk[n] = (double)h[1][i];
        ++n;
      }
    nkeep = n;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int n = nkeep;
    const double sp = cgl_np_pairwise_sum(pk, n), sq = cgl_np_pairwise_sum(qk, n);
    for (int i = 0; i < n; ++i) {
      const double p = pk[i] / sp, q = qk[i] / sq;
      // scipy.special.rel_entr: p log(p / q) (p > 0, q > 0); 0 (p == 0, q >= 0); inf otherwise
      pk[i] = (p > 0.0 && q > 0.0) ? p * log(p / q) : (p == 0.0 && q >= 0.0 ? 0.0 : __longlong_as_double(0x7ff0000000000000LL));
    }
    a.kl[0] = cgl_np_pairwise_sum(pk, n);
  }
}

extern "C" {

int cgl_kl_score(const float* real, int64_t nr, int64_t real_stride, const float* gen, int64_t ng, int64_t gen_stride,
                 int bins, double lo0, double hi0, double lo1, double hi1, int* counts, double* kl, void* stream) {
  CGL_BATCH_GUARD();
  if (!real || !gen || nr < 0 || ng < 0 || real_stride < 1 || gen_stride < 1 || bins < 1 || bins > CGL_HIST_MAXB ||
      !(hi0 > lo0) || !(hi1 > lo1) || (!counts && !kl))
    return CGL_E_ARG;
  CglKlArgs a;
  a.real = real; a.nr = nr; a.sr = real_stride;
  a.gen = gen; a.ng = ng; a.sg = gen_stride;
  a.bins = bins; a.lo0 = lo0; a.hi0 = hi0; a.lo1 = lo1; a.hi1 = hi1;
  a.counts = counts; a.kl = kl;
  hipLaunchKernelGGL(cgl_hist2d_kl_k, dim3(1), dim3(1024), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

}  // extern "C"
