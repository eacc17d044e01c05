"""16-bit GEMM operands (cgl_gan_config.gemm_dtype, BASELINE config 5: MD-GAN, bs512, fp16).

The reference has no 16-bit arithmetic, so this path's parity is UNPINNED.  The HIP
round is compared with two fp64 oracle rounds from the same state and inputs:
  * ``exact``: the reference arithmetic in fp64 -- the 16-bit error itself, bounded loosely (0.2
    relative for bf16, 0.05 for f16: a sanity bound, not a parity claim);
  * ``emu``: the same with the HIP path's rounding restated (oracle.gan_oracle._LowpLinear: every
    GEMM operand rounded to the 16-bit type, exact products, wide accumulation; the D output
    layer in full precision as the HIP loss head computes it).  The HIP path cannot match ``emu``
    to fp32 level: its fp32 activations and the oracle's fp64 ones round to different 16-bit
    neighbours at a few elements per GEMM, and BatchNorm backward amplifies those differences
    layer by layer (tools/lowp_diag.py).  What is required: the losses within 1e-4; every
    other tensor at most 0.1 (forward, D update) / 0.35 (G gradients) of its distance to
    ``exact`` -- a wrong fragment layout or a missed rounding would put the HIP result at or beyond
    the 16-bit error itself (ratio >= 1).
Linear biases that feed a BatchNorm have an analytically zero gradient (pure rounding noise) and
are skipped.  Without loss scaling, f16 G gradients below fp16's normal range (6.1e-5) lose
precision or flush, so for unscaled f16 only the forward, the losses and the D update are judged;
with dynamic loss scaling (``loss_scale``, GradScaler semantics) the G gradients are judged too,
against the emulation run with the same static scale (``test_lowp_scaled_round``), and the scaler's
skip / backoff / growth bookkeeping is checked on rounds built to overflow or not
(``test_loss_scale_*``).
"""
import copy

import pytest
import torch

from parity_helpers import feed, g_params, inputs, make_pair, oracle_round64, rel, rel_scalar, to_double

pytestmark = pytest.mark.gpu

DT = {"bf16": torch.bfloat16, "f16": torch.float16}
EXACT_TOL = {"bf16": 0.2, "f16": 0.05}
BN_FED_BIAS = ("model.2.bias", "model.5.bias", "model.8.bias")


@pytest.fixture(autouse=True)
def _threads():
    n = torch.get_num_threads()
    torch.set_num_threads(8)
    yield
    torch.set_num_threads(n)


@pytest.mark.parametrize("kind,B,dtype", [("mdgan", 512, "bf16"), ("mdgan", 512, "f16"), ("capgan", 256, "bf16")])
def test_lowp_round(kind, B, dtype):
    _lowp_round(kind, B, dtype, 0.0)


@pytest.mark.parametrize("kind,B", [("mdgan", 512), ("capgan", 256)])
def test_lowp_scaled_round(kind, B):
    """f16 with dynamic loss scaling at torch's default initial scale (2^16): no overflow at this
    scale, so the round equals the emulation run with the same static scale -- G gradients judged."""
    _lowp_round(kind, B, "f16", 65536.0)


def _lowp_round(kind, B, dtype, scale):
    srv, workers, step = make_pair(kind, B, gemm_dtype=dtype, loss_scale=scale)
    srv64, workers64 = copy.deepcopy(srv), copy.deepcopy(workers)
    to_double(srv64, workers64)
    emu, wemu = copy.deepcopy(srv64), copy.deepcopy(workers64)
    emu.G.lowp = (DT[dtype], None)
    if scale:
        emu.loss_scale = scale
    for w in wemu:
        w.D.lowp = (DT[dtype], w.D.spec[-2][1] if w.D.spec[-1][0] == "sigmoid" else w.D.spec[-1][1])
        if scale:
            w.loss_scale = scale
    z1, z2, reals = inputs(kind, B, B, 1, seed=11)
    feed(step, z1, z2, reals)
    step.run()
    torch.cuda.synchronize()
    st = step.stats()
    rx = oracle_round64(kind, srv64, workers64, z1, z2, reals)
    re = oracle_round64(kind, emu, wemu, z1, z2, reals)
    out = step.g_output().cpu()
    fail = []
    for key, ek, xk in (("d_loss", re["d_losses"][0], rx["d_losses"][0]), ("g_loss", re["g_losses"][0], rx["g_losses"][0])):
        got = st["d_loss"][0] if key == "d_loss" else st["g_loss"]
        if rel_scalar(got, ek) > 1e-4 or rel_scalar(got, xk) > EXACT_TOL[dtype]:
            fail.append((key, got, float(ek), float(xk)))

    def judge(name, got, e_ref, x_ref, ratio):
        ee, ex = rel(got, e_ref), rel(got, x_ref)
        if ex > EXACT_TOL[dtype] or ee > ratio * ex + 1e-6:
            fail.append((name, ee, ex))

    fwd_ratio = 0.1 if dtype == "bf16" else 0.25   # f16's exact error is ~8x smaller, the flips are not
    judge("Xd", out[:B], re["Xd"].reshape(B, -1), rx["Xd"].reshape(B, -1), fwd_ratio)
    judge("Xg", out[B:], re["Xg"].reshape(B, -1), rx["Xg"].reshape(B, -1), fwd_ratio)
    # Adam's first step maps each D gradient to about +-lr whatever its size, so a D element whose
    # gradient is near zero takes opposite steps under any two roundings; with the CE head (capgan)
    # a few such flips dominate the D update's difference and, through the updated D, the G
    # gradients' -- there the HIP path is only required to be no farther from ``emu`` than from
    # ``exact`` (D) / 0.6 of it (G)
    # (f16: its exact error is ~8x smaller than bf16's while the neighbour flips are not -- as fwd_ratio)
    d_ratio, g_ratio = (fwd_ratio, 0.35 if dtype == "bf16" else 0.5) if kind == "mdgan" else (1.1, 0.6)
    for k, v in step.d_views.items():
        judge("D " + k, v, wemu[0].D.params[k], workers64[0].D.params[k], d_ratio)
    pe, px = g_params(emu.G), g_params(srv64.G)
    for k, v in step.g_grad_views.items():
        if k not in BN_FED_BIAS and (dtype == "bf16" or scale):
            judge("dG " + k, v, pe[k].grad, px[k].grad, g_ratio)
    if scale:
        assert st["loss_scale"] == [scale, scale] and st["last_skipped"] == [0, 0], st
    assert not fail, fail


def _scaled_step(scale, interval=2000):
    srv, workers, step = make_pair("mdgan", 512, gemm_dtype="f16", loss_scale=scale,
                                   scale_growth_interval=interval)
    z1, z2, reals = inputs("mdgan", 512, 512, 1, seed=11)
    feed(step, z1, z2, reals)
    return step


def test_loss_scale_overflow_skips_step():
    """A scale of 2^40 overflows the f16 gradient operands (the D-step and G-loss dlogits are ~1e-3):
    both models' weight gradients turn non-finite, both Adam steps are skipped (parameters and moments
    unchanged), the gradients are left unscaled, and the next round's prologue halves both scales."""
    step = _scaled_step(2.0 ** 40)
    before = [t.clone() for t in (step.g_params, step.g_m, step.g_v, step.d_params, step.d_m, step.d_v)]
    step.run()
    torch.cuda.synchronize()
    st = step.stats()
    after = (step.g_params, step.g_m, step.g_v, step.d_params, step.d_m, step.d_v)
    for b, a in zip(before, after):
        assert torch.equal(b, a)
    assert not torch.isfinite(step.g_grads).all() and not torch.isfinite(step.d_grads).all()
    assert st["loss_scale"] == [2.0 ** 40, 2.0 ** 40] and st["last_skipped"] == [1, 1] and st["skipped"] == [1, 1], st
    step.run()
    torch.cuda.synchronize()
    st = step.stats()
    assert st["loss_scale"] == [2.0 ** 39, 2.0 ** 39] and st["skipped"] == [2, 2], st
    for b, a in zip(before, after):
        assert torch.equal(b, a)


def test_loss_scale_growth_and_step_count():
    """No overflow at 2^10: every step is taken and the scale doubles after `interval` clean rounds
    (GradScaler.update applied by the next round's prologue)."""
    step = _scaled_step(1024.0, interval=2)
    seen = []
    for _ in range(5):
        step.run()
        torch.cuda.synchronize()
        st = step.stats()
        assert st["last_skipped"] == [0, 0], st
        seen.append(st["loss_scale"][0])
        assert st["loss_scale"][0] == st["loss_scale"][1]
    # prologue of round r applies round r-1's update: growth 1, 2 -> x2, 1, 2 -> x2
    assert seen == [1024.0, 1024.0, 2048.0, 2048.0, 4096.0], seen
    assert st["skipped"] == [0, 0]
