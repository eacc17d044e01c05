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
are skipped.  fp16 has no loss scaling: G gradients below fp16's normal range (6.1e-5) lose
precision or flush, so for f16 only the forward, the losses and the D update are judged (bf16,
with fp32's exponent range, is the config-5 variant bench.py reports).
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
    srv, workers, step = make_pair(kind, B, gemm_dtype=dtype)
    srv64, workers64 = copy.deepcopy(srv), copy.deepcopy(workers)
    to_double(srv64, workers64)
    emu, wemu = copy.deepcopy(srv64), copy.deepcopy(workers64)
    emu.G.lowp = (DT[dtype], None)
    for w in wemu:
        w.D.lowp = (DT[dtype], w.D.spec[-2][1] if w.D.spec[-1][0] == "sigmoid" else w.D.spec[-1][1])
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
    d_ratio, g_ratio = (fwd_ratio, 0.35) if kind == "mdgan" else (1.1, 0.6)
    for k, v in step.d_views.items():
        judge("D " + k, v, wemu[0].D.params[k], workers64[0].D.params[k], d_ratio)
    pe, px = g_params(emu.G), g_params(srv64.G)
    for k, v in step.g_grad_views.items():
        if k not in BN_FED_BIAS and dtype == "bf16":
            judge("dG " + k, v, pe[k].grad, px[k].grad, g_ratio)
    assert not fail, fail
