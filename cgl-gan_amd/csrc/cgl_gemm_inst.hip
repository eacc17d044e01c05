// GEMM-instantiation translation unit of libcglgan_hip: compiled once per part (-DCGL_GEMM_PART=1..4), each
// time defining that part's instances of cgl_gemm_f32 / cgl_gemm_pro / cgl_gemm_adam (cgl_gemm_inst.h).
// Only device code and these kernels are compiled here; cgl_runtime.hip declares and launches them.
#define CGL_GEMM_PART_TU 1
#include "cgl_gemm.hip"
#include "cgl_kernels.hip"
#include "cgl_round.h"

#define CGL_INST_PREFIX template
#include "cgl_gemm_inst.h"
