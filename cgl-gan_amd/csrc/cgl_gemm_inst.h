// Every instance of the GEMM kernel templates the runtime launches, split into the parts compiled by the
// cgl_gemm_inst.hip translation units (make builds them in parallel).  Included with
//   CGL_INST_PREFIX = "extern template" (cgl_runtime.hip: declarations only) or
//   CGL_INST_PREFIX = "template" + CGL_GEMM_PART = p (cgl_gemm_inst.hip: the definitions of part p).
#ifndef CGL_INST_PREFIX
#error "define CGL_INST_PREFIX"
#endif
#ifdef CGL_GEMM_PART
#define CGL_IN_PART(p) (CGL_GEMM_PART == (p))
#else
#define CGL_IN_PART(p) 1
#endif

#define CGL_INST_F32(TM, TN, SK, DT, ABN) \
  CGL_INST_PREFIX __global__ void cgl_gemm_f32<TM, TN, SK, DT, ABN>(const CglGemmDesc* __restrict__, int, int, int, int, \
                                                                     const int* __restrict__, int);
#define CGL_INST_ARG(TM, TN) \
  CGL_INST_PREFIX __global__ void cgl_gemm_f32_arg<TM, TN>(const CglGemmDesc);
#define CGL_INST_PRO(TM, TN)                                                                                    \
  CGL_INST_PREFIX __global__ void cgl_gemm_pro<TM, TN>(const CglGemmDesc* __restrict__, int, const int* __restrict__, int, CglBeginArgs, float*, \
                                                       long, unsigned long long, int*, int, int, int,            \
                                                       unsigned long long, CglOpPack);
#define CGL_INST_ADAM(TM, TN)                                                                                   \
  CGL_INST_PREFIX __global__ void cgl_gemm_adam<TM, TN>(const CglGemmDesc* __restrict__, int, int, CglAdamArgs,  \
                                                        CglStepState*, int);

#if CGL_IN_PART(1)   // the default fp32 plan
CGL_INST_F32(1, 1, false, CGL_DTYPE_F32, 0)
CGL_INST_F32(2, 2, false, CGL_DTYPE_F32, 0)
CGL_INST_PRO(1, 1)
CGL_INST_PRO(2, 2)
#endif
#if CGL_IN_PART(2)   // fp32 split-K, the forward BatchNorm operand transform, the single-op (by-value) form
CGL_INST_ARG(1, 1)
CGL_INST_ARG(2, 2)
CGL_INST_F32(1, 1, true, CGL_DTYPE_F32, 0)
CGL_INST_F32(2, 2, true, CGL_DTYPE_F32, 0)
CGL_INST_F32(1, 1, false, CGL_DTYPE_F32, 1)
CGL_INST_F32(2, 2, false, CGL_DTYPE_F32, 1)
#endif
#if CGL_IN_PART(3)   // the backward BatchNorm operand transform, f16 operands
CGL_INST_F32(1, 1, false, CGL_DTYPE_F32, 2)
CGL_INST_F32(2, 2, false, CGL_DTYPE_F32, 2)
CGL_INST_F32(1, 1, true, CGL_DTYPE_F16, 0)
CGL_INST_F32(2, 2, true, CGL_DTYPE_F16, 0)
CGL_INST_F32(1, 1, false, CGL_DTYPE_F16, 0)
CGL_INST_F32(2, 2, false, CGL_DTYPE_F16, 0)
#endif
#if CGL_IN_PART(4)   // bf16 operands, the weight-gradient + Adam fusion
CGL_INST_F32(1, 1, true, CGL_DTYPE_BF16, 0)
CGL_INST_F32(2, 2, true, CGL_DTYPE_BF16, 0)
CGL_INST_F32(1, 1, false, CGL_DTYPE_BF16, 0)
CGL_INST_F32(2, 2, false, CGL_DTYPE_BF16, 0)
CGL_INST_ADAM(1, 1)
CGL_INST_ADAM(2, 2)
#endif

#undef CGL_INST_F32
#undef CGL_INST_ARG
#undef CGL_INST_PRO
#undef CGL_INST_ADAM
#undef CGL_IN_PART
