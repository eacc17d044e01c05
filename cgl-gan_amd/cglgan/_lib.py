"""ctypes binding of libcglgan_hip.so (the C ABI declared in include/cglgan.h).

The library is the product: there is no Python or CPU fallback.  If the shared object is
missing, importing this module raises immediately (build it with ``make -C cgl-gan_amd`` or
``python -c "import __graft_entry__ as g; g.build()"``).
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CGL_LIB_PATH") or os.path.join(os.path.dirname(_HERE), "lib", "libcglgan_hip.so")

MAX_LAYERS = 8
LOSS_CE2, LOSS_BCE = 0, 1
WEIGHT_CAPGAN, WEIGHT_MEAN, WEIGHT_MIX_SINGLE, WEIGHT_MIX_DOUBLE, WEIGHT_CGLGAN = 0, 1, 2, 3, 4
PHASE_ALL, PHASE_A, PHASE_B = 0, 1, 2
DTYPE_F32, DTYPE_F16, DTYPE_BF16 = 0, 1, 2
MODEL_G, MODEL_D = 0, 1

# every symbol include/cglgan.h declares (checked by tests/test_lib_exports.py)
EXPORTS = [
    "cgl_gan_param_count", "cgl_gan_param_tensor", "cgl_gan_running_count", "cgl_gan_workspace_bytes",
    "cgl_gan_create", "cgl_gan_destroy", "cgl_gan_reset", "cgl_gan_sync_params", "cgl_gan_sync_params_d", "cgl_gan_gemm_trace", "cgl_gan_run", "cgl_gan_run_graph", "cgl_gan_run_graph_rounds", "cgl_gan_prepare_graph_rounds",
    "cgl_gan_alpha_scale", "cgl_gan_exchange_mode", "cgl_gan_gather_buffers",
    "cgl_gan_exchange_buffer", "cgl_gan_tensor", "cgl_gan_read_stats",
    "cgl_gan_plan_info", "cgl_gan_launch_count", "cgl_gan_launch_info", "cgl_gan_launch_one", "cgl_gan_profile", "cgl_linear_fwd", "cgl_linear_bwd_data", "cgl_linear_bwd_weight", "cgl_adam_step",
    "cgl_normal_fill", "cgl_op_workspace_bytes", "cgl_version", "cgl_act_fwd", "cgl_act_bwd", "cgl_bn1d_fwd",
    "cgl_bn1d_bwd",
    # conv GAN path (model/lsgan.py)
    "cgl_conv3x3_workspace_bytes", "cgl_conv3x3_fwd", "cgl_conv3x3_bwd_data", "cgl_conv3x3_bwd_weight",
    "cgl_conv3x3_bwd_weight_bnin", "cgl_conv3x3_bwd_weight_actdrop",
    "cgl_bn2d_workspace_bytes", "cgl_bn2d_fwd", "cgl_bn2d_bwd", "cgl_act_drop_bwd", "cgl_act_drop_bwd_colsum", "cgl_colsum_finalize", "cgl_dropout2d_mask", "cgl_dropout2d_masks",
    "cgl_nchw_to_nhwc", "cgl_nhwc_to_nchw", "cgl_dense1_bwd_data_nhwc", "cgl_dense1_fwd_nhwc", "cgl_dense1_head_nhwc", "cgl_adv_loss", "cgl_adam_multi", "cgl_dense_workspace_bytes",
    "cgl_dense_fwd", "cgl_dense_bwd_data", "cgl_dense_bwd_weight", "cgl_gather_rows", "cgl_weights_scale",
    "cgl_conv_packed_floats", "cgl_conv_pack_multi", "cgl_conv_batch_begin", "cgl_conv_batch_end", "cgl_conv_wgrad_defer_begin", "cgl_conv_wgrad_defer_end", "cgl_conv_wgrad_defer_counters", "cgl_conv3x3_bias_by_colsum", "cgl_conv3x3_fwd_packed", "cgl_conv3x3_bwd_data_packed",
    "cgl_dense_fwd_packed", "cgl_dense_bwd_data_packed", "cgl_conv3x3_stat_chunks", "cgl_conv3x3_fwd_packed_stats",
    "cgl_bn2d_fwd_stats", "cgl_bn2d_fwd_stats_coef", "cgl_conv3x3_fwd_packed_bnin", "cgl_bn2d_stats_scratch_bytes", "cgl_linear_desc_bytes", "cgl_linear_prepare", "cgl_linear_prepare_gather", "cgl_linear_prepare_wgrad_nhwc",
    "cgl_linear_launch", "cgl_conv3x3_bwd_stat_chunks", "cgl_conv3x3_bwd_data_packed_stats", "cgl_conv3x3_bwd_data_stats", "cgl_bn2d_bwd_stats",
    "cgl_normal_fill_dev", "cgl_dropout2d_masks_dev", "cgl_adam_multi_dev", "cgl_sample_rows_dev", "cgl_counters_add",
    # evaluation (CGLGAN/2DMG/main.py plot_2d KL score)
    "cgl_kl_score",
]

LOSS_OP_CE2, LOSS_OP_BCE, LOSS_OP_MSE, LOSS_OP_BCE_LOGIT = 0, 1, 2, 3


class MlpSpec(ctypes.Structure):
    _fields_ = [("n_layers", ctypes.c_int), ("dims", ctypes.c_int * (MAX_LAYERS + 1)),
                ("bn", ctypes.c_int * MAX_LAYERS)]


class GanConfig(ctypes.Structure):
    _fields_ = [("g", MlpSpec), ("d", MlpSpec), ("batch", ctypes.c_int), ("batch_real", ctypes.c_int),
                ("epoch", ctypes.c_int), ("loss", ctypes.c_int), ("weighting", ctypes.c_int),
                ("n_workers", ctypes.c_int), ("rank", ctypes.c_int), ("exchange_layer", ctypes.c_int),
                ("lr_g", ctypes.c_double), ("lr_d", ctypes.c_double), ("beta1", ctypes.c_double),
                ("beta2", ctypes.c_double), ("adam_eps", ctypes.c_double), ("bn_eps", ctypes.c_double),
                ("bn_momentum", ctypes.c_double), ("slope", ctypes.c_float), ("seed", ctypes.c_ulonglong),
                ("gen_z", ctypes.c_int), ("sample_n", ctypes.c_int), ("gemm_dtype", ctypes.c_int),
                ("loss_scale", ctypes.c_float), ("scale_growth_interval", ctypes.c_int)]


class GanBuffers(ctypes.Structure):
    _fields_ = [("g_params", ctypes.c_void_p), ("g_grads", ctypes.c_void_p), ("g_m", ctypes.c_void_p),
                ("g_v", ctypes.c_void_p), ("g_running", ctypes.c_void_p), ("d_params", ctypes.c_void_p),
                ("d_grads", ctypes.c_void_p), ("d_m", ctypes.c_void_p), ("d_v", ctypes.c_void_p),
                ("z", ctypes.c_void_p), ("real", ctypes.c_void_p), ("real_idx", ctypes.c_void_p),
                ("losses_all", ctypes.c_void_p), ("workspace", ctypes.c_void_p),
                ("workspace_bytes", ctypes.c_int64)]


class ConvPackJob(ctypes.Structure):
    _fields_ = [("W", ctypes.c_void_p), ("Wp", ctypes.c_void_p), ("h", ctypes.c_int), ("w", ctypes.c_int),
                ("cin", ctypes.c_int), ("cout", ctypes.c_int), ("stride", ctypes.c_int), ("up", ctypes.c_int),
                ("ks", ctypes.c_int), ("dir", ctypes.c_int)]


class LinearLaunch(ctypes.Structure):
    _fields_ = [("tm", ctypes.c_int), ("grid", ctypes.c_int), ("shmem", ctypes.c_int), ("flags", ctypes.c_int)]


class GanStats(ctypes.Structure):
    _fields_ = [("round", ctypes.c_int), ("d_loss", ctypes.c_float * 8), ("d_real", ctypes.c_float * 8),
                ("d_fake", ctypes.c_float * 8), ("g_loss", ctypes.c_float), ("alpha", ctypes.c_float),
                ("F", ctypes.c_float), ("lambda_", ctypes.c_float), ("bn_batches", ctypes.c_longlong),
                ("loss_scale", ctypes.c_float * 2), ("last_skipped", ctypes.c_int * 2), ("skipped", ctypes.c_int * 2)]


def _hip_runtimes():
    """Paths of every libamdhip64 mapped into this process (Linux)."""
    try:
        with open("/proc/self/maps") as f:
            return {ln.split()[-1] for ln in f if "libamdhip64" in ln and "/" in ln}
    except OSError:
        return set()


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libcglgan_hip.so not built ({LIB_PATH}); run `make -C cgl-gan_amd` "
                          "(there is no CPU fallback)")
    # torch first: its HIP runtime (libamdhip64.so.7 in torch/lib) must be the one the library binds to, so that
    # both share one device context, the streams torch hands us and torch.cuda.graph capture.  Loaded the other
    # way round, the dynamic loader resolves our libamdhip64.so.7 to /opt/rocm's copy and torch later maps its own:
    # two runtimes in one process, and every library call fails (hipErrorNoDevice, seen on the GPU box when a test
    # module imported cglgan before torch).
    import torch  # noqa: F401
    lib = ctypes.CDLL(LIB_PATH)
    rts = _hip_runtimes()
    if len(rts) > 1:
        raise ImportError(f"two HIP runtimes are mapped into this process ({sorted(rts)}): import torch before "
                          "loading libcglgan_hip.so by any other path")
    P = ctypes.POINTER
    vp, i64, ci, cf, cd = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float, ctypes.c_double
    sig = {
        "cgl_gan_param_count": (i64, [P(GanConfig), ci]),
        "cgl_gan_param_tensor": (ci, [P(GanConfig), ci, ci, P(i64), P(ci), P(ci), P(ci), P(ci)]),
        "cgl_gan_running_count": (i64, [P(GanConfig)]),
        "cgl_gan_workspace_bytes": (i64, [P(GanConfig)]),
        "cgl_gan_create": (ci, [P(GanConfig), P(GanBuffers), P(vp)]),
        "cgl_gan_destroy": (ci, [vp]),
        "cgl_gan_reset": (ci, [vp, P(cf), vp]),
        "cgl_gan_sync_params": (ci, [vp, vp]),
        "cgl_gan_sync_params_d": (ci, [vp, vp]),
        "cgl_gan_gemm_trace": (i64, [vp, vp, i64]),
        "cgl_gan_run": (ci, [vp, ci, vp]),
        "cgl_gan_run_graph": (ci, [vp, ci, vp]),
        "cgl_gan_run_graph_rounds": (ci, [vp, ci, vp]),
        "cgl_gan_prepare_graph_rounds": (ci, [vp, ci, vp]),
        "cgl_gan_alpha_scale": (ci, [vp, vp]),
        "cgl_gan_exchange_mode": (ci, [vp, ci]),
        "cgl_gan_gather_buffers": (ci, [vp, vp, vp, vp]),
        "cgl_gan_exchange_buffer": (ci, [vp, P(vp), P(i64)]),
        "cgl_gan_tensor": (ci, [vp, ci, P(vp), P(i64)]),
        "cgl_gan_read_stats": (ci, [vp, P(GanStats), vp]),
        "cgl_gan_plan_info": (ci, [vp, ci, P(ci), P(ci), P(ctypes.c_double)]),
        "cgl_gan_launch_count": (ci, [vp, ci]),
        "cgl_gan_launch_info": (ci, [vp, ci, ci, P(ci), P(cd), P(ci)]),
        "cgl_gan_launch_one": (ci, [vp, ci, ci, vp]),
        "cgl_gan_profile": (ci, [vp, ci, vp, P(ctypes.c_float), ci]),
        "cgl_linear_fwd": (ci, [vp, vp, vp, vp, ci, ci, ci, ci, cf, vp, i64, vp]),
        "cgl_linear_bwd_data": (ci, [vp, vp, vp, ci, ci, ci, vp, i64, vp]),
        "cgl_linear_bwd_weight": (ci, [vp, vp, vp, vp, ci, ci, ci, vp, i64, vp]),
        "cgl_adam_step": (ci, [vp, vp, vp, vp, i64, ci, cd, cd, cd, cd, vp, i64, vp]),
        "cgl_normal_fill": (ci, [vp, i64, ctypes.c_ulonglong, ci, ci, vp]),
        "cgl_act_fwd": (ci, [vp, i64, ci, cf, vp, vp]),
        "cgl_act_bwd": (ci, [vp, vp, i64, ci, cf, vp, vp]),
        "cgl_bn1d_fwd": (ci, [vp, ci, ci, ci, vp, vp, cd, cd, vp, vp, ci, ci, cf, vp, vp, vp, vp, i64, vp]),
        "cgl_bn1d_bwd": (ci, [vp, vp, vp, ci, ci, vp, vp, vp, ci, cf, vp, vp, vp, vp, i64, vp]),
        "cgl_op_workspace_bytes": (i64, []),
        "cgl_conv3x3_workspace_bytes": (i64, [ci] * 7),
        "cgl_conv3x3_fwd": (ci, [vp, vp, vp, vp] + [ci] * 8 + [cf, vp, vp, i64, vp]),
        "cgl_conv3x3_bwd_data": (ci, [vp, vp, vp] + [ci] * 7 + [vp, i64, vp]),
        "cgl_conv3x3_bwd_weight": (ci, [vp, vp, vp, vp] + [ci] * 7 + [vp, i64, vp]),
        "cgl_conv3x3_bwd_weight_bnin": (ci, [vp, vp, vp, vp] + [ci] * 7 + [vp, ci, ci, ci, cf, vp, i64, vp]),
        "cgl_conv3x3_bwd_weight_actdrop": (ci, [vp, vp, vp, cf, vp, vp, vp] + [ci] * 7 + [vp, i64, vp]),
        "cgl_bn2d_workspace_bytes": (i64, [ci] * 4),
        "cgl_bn2d_fwd": (ci, [vp, ci, ci, ci, ci, vp, vp, cd, cd, vp, vp, ci, ci, cf, vp, vp, vp, vp, vp, i64, vp]),
        "cgl_bn2d_bwd": (ci, [vp, vp, vp, ci, ci, ci, ci, vp, vp, vp, cf, vp, vp, vp, vp, vp, vp, ci, vp, vp, i64,
                              vp]),
        "cgl_act_drop_bwd": (ci, [vp, vp, vp, ci, ci, ci, cf, ci, vp, vp]),
        "cgl_act_drop_bwd_colsum": (ci, [vp, vp, vp, ci, ci, ci, cf, ci, vp, vp, vp]),
        "cgl_colsum_finalize": (ci, [vp, ci, ci, vp, vp]),
        "cgl_dropout2d_mask": (ci, [vp, ci, ci, cd, ctypes.c_ulonglong, ctypes.c_ulonglong, vp]),
        "cgl_dropout2d_masks": (ci, [ci, P(vp), P(ci), P(ci), cd, ctypes.c_ulonglong, P(ctypes.c_ulonglong), vp]),
        "cgl_nchw_to_nhwc": (ci, [vp, vp, ci, ci, ci, vp]),
        "cgl_dense1_bwd_data_nhwc": (ci, [vp, vp, vp, ci, ci, ci, vp]),
        "cgl_dense1_fwd_nhwc": (ci, [vp, vp, vp, vp, vp, ci, ci, ci, vp]),
        "cgl_nhwc_to_nchw": (ci, [vp, vp, ci, ci, ci, vp]),
        "cgl_adv_loss": (ci, [vp, ci, ci, ci, ci, cd, vp, vp, vp, vp]),
        "cgl_dense1_head_nhwc": (ci, [vp, vp, vp, vp, vp, vp, vp, ci, ci, ci, ci, ci, ci, cd, vp, vp, ci, cd, vp, vp,
                                      ci, vp, vp]),
        "cgl_dense_workspace_bytes": (i64, [ci] * 3),
        "cgl_dense_fwd": (ci, [vp, vp, vp, vp, ci, ci, ci, ci, cf, vp, i64, vp]),
        "cgl_dense_bwd_data": (ci, [vp, vp, vp, ci, ci, ci, vp, i64, vp]),
        "cgl_dense_bwd_weight": (ci, [vp, vp, vp, vp, ci, ci, ci, vp, i64, vp]),
        "cgl_conv_packed_floats": (i64, [ci] * 8),
        "cgl_conv_pack_multi": (ci, [ci, P(ConvPackJob), vp]),
        "cgl_conv_batch_begin": (ci, [vp]),
        "cgl_conv_batch_end": (ci, [vp]),
        "cgl_conv3x3_bias_by_colsum": (ci, [ci, ci, ci, ci, ci, ci, ci]),
        "cgl_conv_wgrad_defer_begin": (ci, []),
        "cgl_conv_wgrad_defer_end": (ci, [vp]),
        "cgl_conv_wgrad_defer_counters": (ci, [vp, ci, ci, vp, ci]),
        "cgl_conv3x3_fwd_packed": (ci, [vp, vp, vp, vp] + [ci] * 8 + [cf, vp, vp, i64, vp]),
        "cgl_conv3x3_bwd_data_packed": (ci, [vp, vp, vp, vp] + [ci] * 7 + [vp, i64, vp]),
        "cgl_conv3x3_stat_chunks": (i64, [ci] * 8),
        "cgl_conv3x3_fwd_packed_stats": (ci, [vp, vp, vp, vp] + [ci] * 8 + [cf, vp, ci, vp, vp, vp, i64, vp]),
        "cgl_bn2d_fwd_stats": (ci, [vp, ci, vp, ci, ci, ci, ci, vp, vp, cd, cd, vp, vp, ci, cf, vp, vp, vp, vp, vp, vp, i64,
                                    vp]),
        "cgl_bn2d_fwd_stats_coef": (ci, [vp, ci, vp, ci, ci, ci, ci, vp, vp, cd, cd, vp, vp, ci, cf, vp, vp, vp, vp, vp, ci,
                                         vp, vp, i64, vp]),
        "cgl_conv3x3_fwd_packed_bnin": (ci, [vp, vp, vp, vp] + [ci] * 8 + [cf, vp, ci, vp, vp, ci, ci, cf, vp, vp, i64,
                                                                      vp]),
        "cgl_bn2d_stats_scratch_bytes": (i64, [ci, ci]),
        "cgl_linear_desc_bytes": (i64, []),
        "cgl_conv3x3_bwd_stat_chunks": (i64, [ci] * 8),
        "cgl_conv3x3_bwd_data_packed_stats": (ci, [vp, vp, vp] + [ci] * 8 + [vp, vp, vp, vp, ci, vp, cf, vp, i64, vp]),
        "cgl_conv3x3_bwd_data_stats": (ci, [vp, vp, vp] + [ci] * 8 + [vp, vp, vp, vp, ci, vp, cf, vp, i64, vp]),
        "cgl_bn2d_bwd_stats": (ci, [vp, ci, vp, vp, vp, ci, ci, ci, ci, vp, vp, vp, cf, vp, vp, vp, vp, vp, vp, ci, vp,
                                    vp, vp, i64, vp]),
        "cgl_linear_prepare": (ci, [ci, vp, vp, vp, vp, vp, ci, ci, ci, ci, cf, vp, P(LinearLaunch)]),
        "cgl_linear_prepare_gather": (ci, [vp, vp, vp, vp, vp, ci, ci, ci, ci, cf, vp, P(LinearLaunch)]),
        "cgl_linear_prepare_wgrad_nhwc": (ci, [vp, vp, vp, vp, ci, ci, ci, ci, vp, P(LinearLaunch)]),
        "cgl_linear_launch": (ci, [vp, P(LinearLaunch), vp]),
        "cgl_dense_fwd_packed": (ci, [vp, vp, vp, vp, ci, ci, ci, ci, cf, vp, i64, vp]),
        "cgl_dense_bwd_data_packed": (ci, [vp, vp, vp, ci, ci, ci, vp, i64, vp]),
        "cgl_gather_rows": (ci, [vp, vp, i64, ci, ci, vp, vp]),
        "cgl_weights_scale": (ci, [ci, ci, ci, cf, P(cf), vp, vp, i64, vp, vp]),
        "cgl_kl_score": (ci, [vp, i64, i64, vp, i64, i64, ci, cd, cd, cd, cd, vp, vp, vp]),
        "cgl_adam_multi": (ci, [ci, P(vp), P(vp), P(vp), P(vp), P(i64), ci, cd, cd, cd, cd, vp]),
        "cgl_adam_multi_dev": (ci, [ci, P(vp), P(vp), P(vp), P(vp), P(i64), vp, cd, cd, cd, cd, vp]),
        "cgl_normal_fill_dev": (ci, [vp, i64, ctypes.c_ulonglong, vp, ci, vp]),
        "cgl_dropout2d_masks_dev": (ci, [ci, P(vp), P(ci), P(ci), cd, ctypes.c_ulonglong, P(ctypes.c_ulonglong), vp,
                                         ctypes.c_ulonglong, vp]),
        "cgl_sample_rows_dev": (ci, [vp, ci, ci, ci, ctypes.c_ulonglong, vp, vp, vp, vp]),
        "cgl_counters_add": (ci, [vp, ci, ci, vp]),
        "cgl_version": (ctypes.c_char_p, []),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


# CGL_SYNC_CHECK=1: synchronise the device after every C-ABI call that returns through check() and
# name the call on a device fault (a fault otherwise surfaces at some later call, whenever the runtime
# next polls the queue).  Diagnostics only: it serialises the host with the GPU.
_SYNC_CHECK = os.environ.get("CGL_SYNC_CHECK", "0") == "1"
_SYNC_N = [0]


def check(rc, what="libcglgan_hip"):
    """Turn a non-zero C-ABI return code into RuntimeError (include/cglgan.h conventions)."""
    if rc != 0:
        kinds = {-1: "invalid argument", -2: "bad call order", -3: "buffer too small"}
        raise RuntimeError(f"{what} failed: rc={rc} ({kinds.get(rc, 'hipError')})")
    if _SYNC_CHECK:
        import torch
        if not torch.cuda.is_current_stream_capturing():
            _SYNC_N[0] += 1
            try:
                torch.cuda.synchronize()
            except Exception as e:
                raise RuntimeError(f"CGL_SYNC_CHECK: device fault in or before call #{_SYNC_N[0]} ({what})") from e
    return rc


def version():
    return lib.cgl_version().decode()
