"""The C-ABI library loads on CPU and exports every symbol include/cglgan.h declares.

Only host-side (no-device) entry points are called here: layout / sizing queries and config
validation.  Compute calls need a GPU and live in the ``-m gpu`` tests.
"""
import ctypes
import os
import re

import pytest
import torch

from cglgan import _lib as C
from cglgan import specs
from cglgan.step import _spec
from oracle import gan_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "cglgan.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(cgl_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported():
    decl = declared_symbols()
    assert decl, "no declarations parsed"
    assert sorted(C.EXPORTS) == decl
    for name in decl:
        assert hasattr(C.lib, name), name
    assert C.version().endswith("gfx950")


def test_nm_exports():
    out = os.popen(f"nm -D --defined-only {C.LIB_PATH}").read()
    for name in declared_symbols():
        assert re.search(rf"\bT {name}$", out, re.M), name


def _cfg(g, d, B=64, Br=None, loss=C.LOSS_CE2, epoch=1, n_workers=1, rank=0, xl=-1):
    cfg = C.GanConfig()
    cfg.g, cfg.d = _spec(g), _spec(d)
    cfg.batch, cfg.batch_real, cfg.epoch = B, Br or B, epoch
    cfg.loss, cfg.weighting = loss, 0
    cfg.n_workers, cfg.rank, cfg.exchange_layer = n_workers, rank, xl
    cfg.lr_g = cfg.lr_d = 2e-4
    cfg.beta1, cfg.beta2, cfg.adam_eps = 0.5, 0.999, 1e-8
    cfg.bn_eps, cfg.bn_momentum, cfg.slope = 0.8, 0.1, 0.2
    return cfg


def _layout(cfg, which, n):
    out = []
    for i in range(n):
        off, r, c, l, k = ctypes.c_int64(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        assert C.lib.cgl_gan_param_tensor(ctypes.byref(cfg), which, i, ctypes.byref(off), ctypes.byref(r),
                                          ctypes.byref(c), ctypes.byref(l), ctypes.byref(k)) == 0
        out.append((off.value, r.value, c.value, l.value, k.value))
    assert C.lib.cgl_gan_param_tensor(ctypes.byref(cfg), which, n, None, None, None, None, None) == C_E_ARG
    return out


C_E_ARG = -1


@pytest.mark.parametrize("kind", ["capgan", "mixg", "mdgan", "ring"])
def test_layout_matches_reference_state_dict(kind):
    if kind == "capgan":
        gm, dm = specs.mnist_generator(), specs.mnist_discriminator()
        G, ws = O.build_capgan(1)
        gsd, dsd = G.state_dict(), ws[0].D.state_dict()
        loss = C.LOSS_CE2
    elif kind == "mixg":
        gm, dm = specs.mixgen_worker(1), specs.mnist_discriminator()
        G, ws = O.build_mixg(2)
        gsd, dsd = G.state_dict(), ws[1].D.state_dict()
        loss = C.LOSS_CE2
    elif kind == "mdgan":
        gm, dm = specs.mnist_generator(), specs.mnist_discriminator(sigmoid=True)
        G, ws = O.build_capgan(1, loss="bce")
        gsd, dsd = G.state_dict(), ws[0].D.state_dict()
        loss = C.LOSS_BCE
    else:
        gm, dm = specs.ring_generator(0), specs.ring_discriminator()
        G, ws = O.build_ring(1, 1)
        gsd, dsd = G.state_dict(), ws[0].D.state_dict()
        loss = C.LOSS_BCE
    cfg = _cfg(gm, dm, loss=loss)
    for m, which, sd in ((gm, C.MODEL_G, gsd), (dm, C.MODEL_D, dsd)):
        keys = m.tensor_keys()
        lay = _layout(cfg, which, len(keys))
        total = C.lib.cgl_gan_param_count(ctypes.byref(cfg), which)
        prev_end = 0
        for k, (off, r, c, l, kd) in zip(keys, lay):
            assert k in sd, k
            assert r * c == sd[k].numel(), k
            if kd == 0:
                assert list(sd[k].shape) == [r, c], k
            assert off % 64 == 0 and off >= prev_end
            prev_end = off + r * c
        assert total >= prev_end
    nr = C.lib.cgl_gan_running_count(ctypes.byref(cfg))
    assert nr == sum(((gm.dims[l + 1] + 63) // 64 * 64) * 2 for l in gm.bn_layers())
    assert C.lib.cgl_gan_workspace_bytes(ctypes.byref(cfg)) > 0


def test_config_validation():
    gm, dm = specs.mnist_generator(), specs.mnist_discriminator()
    ok = _cfg(gm, dm)
    assert C.lib.cgl_gan_workspace_bytes(ctypes.byref(ok)) > 0
    bad = _cfg(gm, dm, loss=C.LOSS_BCE)          # BCE needs a 1-unit D head
    assert C.lib.cgl_gan_workspace_bytes(ctypes.byref(bad)) == C_E_ARG
    bad = _cfg(gm, specs.ring_discriminator())   # G output 784 != D input 2
    assert C.lib.cgl_gan_workspace_bytes(ctypes.byref(bad)) == C_E_ARG
    bad = _cfg(gm, dm, epoch=9)
    assert C.lib.cgl_gan_workspace_bytes(ctypes.byref(bad)) == C_E_ARG
    bad = _cfg(gm, dm, n_workers=2, rank=2)
    assert C.lib.cgl_gan_workspace_bytes(ctypes.byref(bad)) == C_E_ARG
    bad = _cfg(gm, dm, xl=5)
    assert C.lib.cgl_gan_workspace_bytes(ctypes.byref(bad)) == C_E_ARG
    okx = _cfg(gm, dm, xl=specs.MIXGEN_HEAD_LAYER, n_workers=4, rank=3)
    assert C.lib.cgl_gan_workspace_bytes(ctypes.byref(okx)) > 0
    # dynamic loss scaling: 16-bit GEMM operands only, one local D step, a power-of-two scale
    def scaled(scale, dt=C.DTYPE_F16, epoch=1, interval=0):
        c = _cfg(gm, dm, epoch=epoch)
        c.gemm_dtype, c.loss_scale, c.scale_growth_interval = dt, scale, interval
        return C.lib.cgl_gan_workspace_bytes(ctypes.byref(c))
    assert scaled(65536.0) > 0 and scaled(1.0, dt=C.DTYPE_BF16) > 0
    assert scaled(65536.0, dt=C.DTYPE_F32) == C_E_ARG
    assert scaled(65536.0, epoch=2) == C_E_ARG
    assert scaled(1000.0) == C_E_ARG and scaled(-2.0) == C_E_ARG and scaled(float("inf")) == C_E_ARG
    assert scaled(1024.0, interval=-1) == C_E_ARG
    # create() rejects null buffers without touching a device
    h = ctypes.c_void_p()
    bufs = C.GanBuffers()
    assert C.lib.cgl_gan_create(ctypes.byref(ok), ctypes.byref(bufs), ctypes.byref(h)) == C_E_ARG


def test_ops_reject_bad_args():
    assert C.lib.cgl_linear_fwd(None, None, None, None, 1, 1, 1, 0, 0.2, None, 0, None) == C_E_ARG
    assert C.lib.cgl_adam_step(None, None, None, None, 1, 1, 1e-3, 0.5, 0.999, 1e-8, None, 0, None) == C_E_ARG
    assert C.lib.cgl_op_workspace_bytes() >= 64


def test_open_launch_batch_refuses_other_launches():
    """while cgl_conv_batch_begin is open on this thread, a non-batchable entry point must not
    launch ahead of the deferred calls: it returns CGL_E_STATE (-2) before touching the device (so this runs
    on CPU).  After _end (an empty batch launches nothing) the same call is validated normally again."""
    E_ARG, E_STATE = -1, -2
    lib = C.lib
    assert lib.cgl_conv_batch_begin(None) == 0
    try:
        assert lib.cgl_conv_batch_begin(None) == E_ARG          # nested begin
        assert lib.cgl_gather_rows(None, None, 0, 1, 4, None, None) == E_STATE
        assert lib.cgl_act_fwd(None, 0, 0, 0.2, None, None) == E_STATE
    finally:
        assert lib.cgl_conv_batch_end(None) == 0
    assert lib.cgl_gather_rows(None, None, 0, 1, 4, None, None) == E_ARG


def test_wgrad_defer_state():
    """cgl_conv_wgrad_defer_begin / _end (round 6): a nested begin and an end without begin return CGL_E_STATE; an
    empty batch launches nothing (so this runs on CPU); cgl_conv_wgrad_defer_counters checks its state and
    arguments; and the Python wrapper refuses a weight gradient without a
    workspace of its own inside the block (its partials would be overwritten before the deferred reduction)."""
    import torch
    from cglgan import conv_ops as O
    E_STATE = -2
    lib = C.lib
    assert lib.cgl_conv_wgrad_defer_end(None) == E_STATE
    assert lib.cgl_conv_wgrad_defer_begin() == 0
    try:
        assert lib.cgl_conv_wgrad_defer_begin() == E_STATE
    finally:
        assert lib.cgl_conv_wgrad_defer_end(None) == 0
    assert lib.cgl_conv_wgrad_defer_end(None) == E_STATE
    # the counters fold: outside a deferral CGL_E_STATE; inside, bad arguments CGL_E_ARG (nothing recorded, so the
    # end launches nothing); the addresses are only checked for null, never dereferenced here
    import ctypes
    fake = ctypes.c_void_p(256)
    assert lib.cgl_conv_wgrad_defer_counters(fake, 3, 1, fake, 0) == E_STATE
    assert lib.cgl_conv_wgrad_defer_begin() == 0
    try:
        assert lib.cgl_conv_wgrad_defer_counters(fake, 0, 1, fake, 0) == -1
        assert lib.cgl_conv_wgrad_defer_counters(fake, 3, 1, fake, 3) == -1
        assert lib.cgl_conv_wgrad_defer_counters(None, 3, 1, fake, 0) == -1
    finally:
        assert lib.cgl_conv_wgrad_defer_end(None) == 0
    with pytest.raises(RuntimeError, match="outside wgrad_defer"):
        O.defer_counters(torch.zeros(3, dtype=torch.int32), torch.zeros(1, dtype=torch.int32), 0)
    O._WDEFER = True          # (the wrapper's check runs before any device work)
    try:
        t = torch.empty(0)
        with pytest.raises(RuntimeError, match="of its own"):
            O.conv3x3_bwd_weight(t, t, t, None, 1, 4, 4, 4, 4)
    finally:
        O._WDEFER = False


def test_one_hip_runtime_whatever_the_import_order():
    """Importing cglgan before torch must not map a second HIP runtime: the library has to bind to torch's
    libamdhip64 (one device context, torch's streams, graph capture).  Round 5 found the GPU suite failing
    with hipErrorNoDevice on every library call when a test module imported cglgan first (/opt/rocm's
    runtime beside torch's); cglgan._lib now loads torch first and refuses a second runtime."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import cglgan\n"
            "from cglgan import _lib\n"
            "rts = _lib._hip_runtimes()\n"
            "assert len(rts) == 1 and 'torch' in next(iter(rts)), rts\n"
            "print('ONE-RUNTIME')\n") % os.path.join(ROOT, "cgl-gan_amd")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ONE-RUNTIME" in r.stdout, r.stdout + r.stderr
