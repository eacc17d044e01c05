"""The oracle's 16-bit GEMM emulation (oracle.gan_oracle._LowpLinear), CPU only: with a rounding
type that rounds nothing (float64 -> float64) one round must equal the plain oracle round exactly
(the custom backward restates F.linear's autograd); with bfloat16 it must differ, by about the
16-bit rounding error."""
import copy

import torch

from oracle import gan_oracle as O
from parity_helpers import inputs, make_pair_oracle_only, oracle_round64, rel_scalar, to_double


def _round(kind, dt):
    srv, workers = make_pair_oracle_only(kind)
    to_double(srv, workers)
    if dt is not None:
        srv.G.lowp = (dt, None)
        for w in workers:
            w.D.lowp = (dt, w.D.spec[-2][1] if w.D.spec[-1][0] == "sigmoid" else w.D.spec[-1][1])
    z1, z2, reals = inputs(kind, 64, 64, 1, seed=3)
    r = oracle_round64(kind, srv, workers, z1, z2, reals)
    return r, {k: v.grad.clone() for k, v in srv.G.params.items()}


def test_lowp_identity_and_bf16():
    for kind in ("capgan", "mdgan"):
        r0, g0 = _round(kind, None)
        r1, g1 = _round(kind, torch.float64)
        assert r0["d_losses"][0] == r1["d_losses"][0] and r0["g_losses"][0] == r1["g_losses"][0]
        for k in g0:
            assert torch.allclose(g0[k], g1[k], rtol=1e-12, atol=1e-15), k
        r2, _ = _round(kind, torch.bfloat16)
        e = rel_scalar(r2["g_losses"][0], r0["g_losses"][0])
        assert 1e-6 < e < 3e-2, e
