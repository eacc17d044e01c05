// Library reference point for the GEMM shapes of one B=256 CAPGAN round: rocBLAS sgemm (fp32)
// device time per call (hipEvent over back-to-back calls).  Tuning aid only.
//   hipcc --offload-arch=gfx950 -O3 tools/rocblas_ref.cpp -lrocblas -o tools/rocblas_ref
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <cstdio>
#include <cstdlib>

struct Shape { const char* name; int layout, M, N, K; };

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 200;
  const Shape shapes[] = {
      {"G0 fwd", 0, 512, 128, 100},  {"G1 fwd", 0, 512, 256, 128},  {"G2 fwd", 0, 512, 512, 256},
      {"G3 fwd", 0, 512, 1024, 512}, {"G4 fwd", 0, 512, 784, 1024}, {"D0 fwd", 0, 512, 512, 784},
      {"D1 fwd", 0, 512, 256, 512},  {"E0 fwd", 0, 256, 512, 784},  {"E1 fwd", 0, 256, 256, 512},
      {"D dQ0", 1, 512, 512, 256},   {"E dS0", 1, 256, 512, 256},   {"E dXg", 1, 256, 784, 512},
      {"G4 dA", 1, 256, 1024, 784},  {"G3 dA", 1, 256, 512, 1024},  {"G2 dA", 1, 256, 256, 512},
      {"G1 dA", 1, 256, 128, 256},   {"D gV1", 2, 256, 512, 512},   {"D gV0", 2, 512, 784, 512},
      {"G gW4", 2, 784, 1024, 256},  {"G gW3", 2, 1024, 512, 256},  {"G gW2", 2, 512, 256, 256},
      {"G gW1", 2, 256, 128, 256},   {"G gW0", 2, 128, 100, 256},
  };
  rocblas_handle h;
  rocblas_create_handle(&h);
  float *A, *B, *C;
  const size_t big = 4u << 20;
  hipMalloc(&A, big * 4);
  hipMalloc(&B, big * 4);
  hipMalloc(&C, big * 4);
  hipMemset(A, 0, big * 4);
  hipMemset(B, 0, big * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const float one = 1.f, zero = 0.f;
  double tot = 0, flop = 0;
  for (const Shape& s : shapes) {
    // row-major C[M][N] = op(A) op(B)  <=>  column-major C^T[N][M] = op(B)^T op(A)^T
    rocblas_operation ta, tb;
    int lda, ldb;
    if (s.layout == 0) {        // A[M][K], B[N][K]: C^T = B . A^T  (col-major: B is K x N -> trans)
      ta = rocblas_operation_transpose; tb = rocblas_operation_none; lda = s.K; ldb = s.K;
    } else if (s.layout == 1) { // A[M][K], B[K][N]
      ta = rocblas_operation_none; tb = rocblas_operation_none; lda = s.N; ldb = s.K;
    } else {                    // A[K][M], B[K][N]
      ta = rocblas_operation_none; tb = rocblas_operation_transpose; lda = s.N; ldb = s.M;
    }
    auto call = [&]() {
      rocblas_sgemm(h, ta, tb, s.N, s.M, s.K, &one, B, lda, A, ldb, &zero, C, s.N);
    };
    for (int i = 0; i < 10; ++i) call();
    hipEventRecord(e0, 0);
    for (int i = 0; i < reps; ++i) call();
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / reps;
    const double f = 2.0 * s.M * s.N * s.K;
    printf("%-8s %d %5d %5d %5d  rocblas %7.2f us  %5.1f TF\n", s.name, s.layout, s.M, s.N, s.K, us, f / us * 1e-6);
    tot += us;
    flop += f;
  }
  printf("rocblas sum: %.1f us for %.3f GFLOP\n", tot, flop * 1e-9);
  return 0;
}
