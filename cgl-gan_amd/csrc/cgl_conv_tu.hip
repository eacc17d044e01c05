// Second translation unit of libcglgan_hip: the conv GAN path of model/lsgan.py (implicit-GEMM
// convolutions, BatchNorm2d, losses, Adam) and the evaluation kernels.  Compiled separately from
// the MLP step (cgl_runtime.hip) so that either side rebuilds alone; shared helpers live in
// cgl_common.h.
#include "cgl_internal.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "cgl_conv.hip"
#include "cgl_eval.hip"
