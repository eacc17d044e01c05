"""Parity of the fused conv-GAN worker round (cglgan.ConvGanStep, model/lsgan.py) with the CPU oracle.

The HIP round and oracle/conv_oracle.py start from the same parameters and consume the same
inputs: z (drawn on device, read back), the real batch, and the Dropout2d scales the round drew
(read back and injected into the oracle).  The oracle runs twice, in float64 (truth) and in float32
(the reference's own CPU arithmetic); per tensor the HIP result must satisfy

    ||hip - fp64|| <= max(STEP_TOL * ||fp64||, 4 * ||fp32 - fp64||)          (1e-5)

i.e. it is within 1e-5 relative of exact, or at least as close to exact as (4x) the reference's
fp32 computation -- the yardstick for quantities that fp32 itself cannot resolve (LeakyReLU
kinks hit by rounding, the analytically-zero gradient of a conv bias that feeds BatchNorm2d).

A bias gradient that is one long cancelling sum (``conv_blocks.8.bias``: the sum of the Tanh-input
gradient over all B x 32 x 32 output pixels) is judged against fp64 by the error bound of the sum
itself, 2 log2(n) eps32 sum|terms| (a tree-ordered fp32 sum of n terms), as a third admissible
bound: the fp32 oracle's own error on such a sum is a matter of luck in its summation order, so a
MORE accurate kernel could fail "4x the fp32 oracle's error" (VERDICT r2, weak #8).
"""
import math

import pytest
import torch

from oracle import conv_oracle as CO

pytestmark = pytest.mark.gpu
STEP_TOL = 1e-5
PRE_BN_BIAS = {"conv_blocks.1.bias", "conv_blocks.5.bias"}   # gradient == 0 analytically


def _err(a, b):
    return float((a.detach().double().cpu() - b.detach().double().cpu()).norm())


def _check(name, hip, o64, o32, fails, tol=STEP_TOL):
    e = _err(hip, o64)
    bound = max(tol * float(o64.detach().double().norm()), 4 * _err(o32, o64), 1e-12)
    if e > bound:
        fails.append(f"{name}: err {e:.3e} > bound {bound:.3e} (fp32 oracle err {_err(o32, o64):.3e})")


EPS32 = 2.0 ** -24
SUM_BIASES = {"conv_blocks.8.bias"}   # bias gradient = one sum over every output pixel


def sum_bound(terms):
    """fp32 error bound of a tree-ordered sum of ``terms`` (float tensor): 2 log2(n) eps sum|t|."""
    n = terms.numel()
    return 2 * math.log2(max(n, 2)) * EPS32 * float(terms.detach().double().abs().sum())


def _check_sum(name, hip, o64, o32, terms, fails):
    e = _err(hip, o64)
    bound = max(STEP_TOL * float(o64.detach().double().norm()), 4 * _err(o32, o64), sum_bound(terms), 1e-12)
    if e > bound:
        fails.append(f"{name}: err {e:.3e} > bound {bound:.3e} (sum bound {sum_bound(terms):.3e})")


SIGN_TOL = 2e-5   # |x| / std below which a GPU LeakyReLU branch may differ from fp64's (parity_helpers)


def _gpu_signs(st, d_calls):
    """The LeakyReLU branch decisions (x > 0, NCHW) the HIP round took, per oracle forward call, and
    where they matter (D: Dropout2d-zeroed channels carry no value and no gradient).  LeakyReLU keeps
    the sign, so y > 0 <=> x > 0 on the stored outputs (G: a1, a2; D: q_k = Dropout2d(LeakyReLU))."""
    B = st.B
    nchw = lambda t: t.permute(0, 3, 1, 2).cpu()
    # a1 / a2 are not stored (or only their Xg half) when the G BatchNorm is folded into the next conv's load
    a1, a2 = nchw(st.g_act("a1") > 0), nchw(st.g_act("a2") > 0)
    signs = {"g1": [a1[:B], a2[:B]], "g2": [a1[B:], a2[B:]]}
    valid = {"g1": [None, None], "g2": [None, None]}
    (dstep, dgl) = d_calls
    signs["dr"] = [nchw(q[:B] > 0) for q in dstep]
    signs["df"] = [nchw(q[B:2 * B] > 0) for q in dstep]
    signs["dg"] = [nchw(q[:B] > 0) for q in dgl]
    valid["dr"] = [nchw(q[:B] != 0) for q in dstep]
    valid["df"] = [nchw(q[B:2 * B] != 0) for q in dstep]
    valid["dg"] = [nchw(q[:B] != 0) for q in dgl]
    return signs, valid


def _check_signs(signs, valid, trace):
    """Every followed branch agrees with the fp64 run's own sign wherever |x| > SIGN_TOL std."""
    worst = 0.0
    for k, ms in signs.items():
        xs = trace[k]
        assert len(xs) == len(ms), k
        for x, m, v in zip(xs, ms, valid[k]):
            bad = (x > 0) != m
            if v is not None:
                bad &= v
            if bool(bad.any()):
                worst = max(worst, float(x[bad].abs().max() / x.std()))
    assert worst <= SIGN_TOL, f"GPU LeakyReLU branch differs from fp64 at |x| = {worst:.2e} std"
    return worst


def _run(B, loss, seed=3, rounds=1, follow_gpu=True):
    """``follow_gpu``: the oracles take the HIP round's LeakyReLU branch decisions (checked against
    the fp64 run's own signs); at B = 256 the G's BatchNorm2d outputs alone hold 2.5e7 LeakyReLU
    inputs, so a few sit within fp32 rounding of 0 and a legitimate flip there moves the conv weight /
    BatchNorm beta gradients far past 1e-5 -- the same treatment as the MLP configs
    (tests/parity_helpers.py MaskedRun)."""
    from cglgan.conv_step import ConvGanStep
    torch.set_num_threads(4)
    st = ConvGanStep(B, loss=loss, seed=seed)
    st.init_default(20211212, 20211213)
    gp0, dp0 = st.G.state_dict(), st.D.state_dict()
    split = lambda sd: ({k: v.cpu() for k, v in sd.items() if "running" not in k and "num_batches" not in k},
                        {k: v.cpu() for k, v in sd.items() if "running" in k or "num_batches" in k})
    gp, gb = split(gp0)
    dp, db = split(dp0)
    o64 = CO.ConvGan(gp, gb, dp, db, loss=loss, dtype=torch.float64)
    o32 = CO.ConvGan(gp, gb, dp, db, loss=loss, dtype=torch.float32)
    g = torch.Generator().manual_seed(seed)
    d_calls = []
    fwd = st._d_forward

    def rec(x, n, groups, masks, **kw):   # keep each D forward call's LeakyReLU outputs (the G-loss pass
        fwd(x, n, groups, masks, **kw)    # reuses the D-step buffers)
        d_calls.append([q[:n].clone() for q in st.q])
    st._d_forward = rec
    outs = []
    for r in range(rounds):
        real = torch.rand(B, 1, 32, 32, generator=g) * 2 - 1
        d_calls.clear()
        st.run(real=real.cuda())
        torch.cuda.synchronize()
        z = st.z.cpu()
        mr = [m[:B].cpu() for m in st.mask_d]
        mf = [m[B:].cpu() for m in st.mask_d]
        mg = [m.cpu() for m in st.mask_g]
        signs, valid, trace = None, None, None
        if follow_gpu:
            signs, valid = _gpu_signs(st, d_calls)
            trace = {}
        r64 = o64.round(z[:B], z[B:], real, mr, mf, mg, signs=signs, trace=trace)
        r32 = o32.round(z[:B], z[B:], real, mr, mf, mg, signs=signs)
        if follow_gpu:
            r64["sign_margin"] = _check_signs(signs, valid, trace)
        outs.append((st.stats(), r64, r32, st.G.grads, st.D.grads))
    return st, o64, o32, outs


@pytest.mark.parametrize("B,loss", [(8, "mse"), (8, "bce"), (256, "mse"), (256, "bce")])
def test_conv_round_parity(B, loss):
    """One round at B = 8 and at the benchmarked B = 256 (bench.py --model lsgan: the same
    geometry, so the same kernel instantiations, tile / split choices and specialised
    Conv2d(64, 1) kernels as the timed round)."""
    st, o64, o32, outs = _run(B, loss)
    s, r64, r32, gg, dg = outs[0]
    fails = []
    for k in ("d_real", "d_fake", "g_loss"):
        _check(k, torch.tensor(s[k]), torch.tensor(r64[k]), torch.tensor(r32[k]), fails)
    _check("Xd", st.xd().permute(0, 3, 1, 2), r64["Xd"], r32["Xd"], fails)
    _check("Xg", st.xg().permute(0, 3, 1, 2), r64["Xg"], r32["Xg"], fails)
    for k, v in r64["g_grads"].items():
        if k in PRE_BN_BIAS:
            continue
        if k in SUM_BIASES:
            _check_sum("G grad " + k, gg[k], v, r32["g_grads"][k], st.dc3g, fails)
            continue
        _check("G grad " + k, gg[k], v, r32["g_grads"][k], fails)
    for k, v in r64["d_grads"].items():
        _check("D grad " + k, dg[k], v, r32["d_grads"][k], fails)
    p0g = {k: v.detach() for k, v in o64.gp.items()}
    for k, v in st.G.params.items():
        if k in PRE_BN_BIAS:   # Adam step of a rounding-noise gradient: bounded by lr
            assert float((v.cpu().double() - o64.gp[k].detach()).abs().max()) <= 2 * 2e-4 + 1e-6, k
            continue
        _check("G param " + k, v, o64.gp[k], o32.gp[k], fails)
    for k, v in st.D.params.items():
        _check("D param " + k, v, o64.dp[k], o32.dp[k], fails)
    for k, v in st.G.running.items():
        _check("G " + k, v, o64.gb[k], o32.gb[k], fails)
    for k, v in st.D.running.items():
        _check("D " + k, v, o64.db[k], o32.db[k], fails)
    assert all(st.G.batches[k] == int(o64.gb[k + ".num_batches_tracked"]) for k in st.G.batches)
    assert all(st.D.batches[k] == int(o64.db[k + ".num_batches_tracked"]) for k in st.D.batches)
    assert not fails, "\n".join(fails)


def test_conv_trajectory_5_rounds():
    """Free-running 5 rounds: losses within 1e-4 relative of the fp64 oracle."""
    B = 8
    st, o64, o32, outs = _run(B, "mse", seed=5, rounds=5, follow_gpu=False)
    for s, r64, r32, _, _ in outs:
        for k in ("d_real", "d_fake", "g_loss"):
            ref = r64[k]
            bound = max(1e-4 * abs(ref), 4 * abs(r32[k] - ref))
            assert abs(s[k] - ref) <= bound, (k, s[k], ref)


def test_conv_round_deterministic():
    """Two replicas with identical state and inputs produce bitwise identical results."""
    from cglgan.conv_step import ConvGanStep
    a, b = ConvGanStep(8, seed=11), ConvGanStep(8, seed=11)
    a.init_default(1, 2)
    b.init_default(1, 2)
    real = torch.rand(8, 1, 32, 32, device="cuda") * 2 - 1
    for _ in range(2):
        a.run(real=real)
        b.run(real=real)
    assert torch.equal(a.G.p, b.G.p) and torch.equal(a.D.p, b.D.p)


@pytest.mark.parametrize("B", [8, 256])
def test_conv_round_graph_replay(B):
    """graph=True: rounds replayed as one captured hipGraph (device-side round state: z round, Dropout2d
    counters, Adam steps, device sampler) equal the same rounds issued op by op, bitwise -- at the
    benchmarked B=256 too (the kernel selection bench.py times)."""
    from cglgan.conv_step import ConvGanStep
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        data = torch.rand(4 * B + 3, 1024, device="cuda", generator=torch.Generator("cuda").manual_seed(3)) * 2 - 1
        a = ConvGanStep(B, seed=21, data=data, graph=True)
        b = ConvGanStep(B, seed=21, data=data, graph=True)
        a.init_default(5, 6)
        b.init_default(5, 6)
        for r in range(4):
            a.run(eager=True)
            b.run()              # round 0 eager, round 1 captured + replayed, rounds 2-3 replays
            assert a.round == b.round == r + 1 and a.G.step == b.G.step and a.D.step == b.D.step
        torch.cuda.synchronize()
    assert b._cuda_graph is not None
    assert torch.equal(a.G.p, b.G.p) and torch.equal(a.D.p, b.D.p)
    assert torch.equal(a.G.m, b.G.m) and torch.equal(a.D.v, b.D.v)
    assert torch.equal(a.lbuf, b.lbuf) and torch.equal(a.x3, b.x3)
    assert torch.equal(a.dstate, b.dstate) and a.dstate[:3].tolist() == [4, 4, 4]
    assert a.G.batches == b.G.batches and a.lam == b.lam
    for k in a.G.running:
        assert torch.equal(a.G.running[k], b.G.running[k]), k
    # the sampler drew real rows of the shard: every image of the last real batch is a row of `data`
    x = b.x3[:B].reshape(B, 1024)
    assert all(bool((data == x[i]).all(dim=1).any()) for i in range(B))


@pytest.mark.parametrize("B", [8, 256])
def test_conv_multi_round_graph(B):
    """ConvGanStep.run_rounds(k): k whole rounds as ONE graph replay equal k single-round replays bitwise (device
    round state, sampler across a pass boundary, Adam steps, running statistics, host bookkeeping)."""
    from cglgan.conv_step import ConvGanStep
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        data = torch.rand(3 * B + 5, 1024, device="cuda", generator=torch.Generator("cuda").manual_seed(7)) * 2 - 1
        a = ConvGanStep(B, seed=23, data=data, graph=True)
        b = ConvGanStep(B, seed=23, data=data, graph=True)
        a.init_default(8, 9)
        b.init_default(8, 9)
        a.run()
        b.run()
        b.prepare_rounds(3)
        for n in (3, 4, 3):
            a.run_rounds(n)
            for _ in range(n):
                b.run()
        torch.cuda.synchronize()
    assert set(a._kgraphs) == {3, 4}
    assert a.round == b.round == 11 and a.G.step == b.G.step and a.D.step == b.D.step
    assert torch.equal(a.G.p, b.G.p) and torch.equal(a.D.p, b.D.p)
    assert torch.equal(a.G.m, b.G.m) and torch.equal(a.D.v, b.D.v)
    assert torch.equal(a.lbuf, b.lbuf) and torch.equal(a.x3, b.x3) and torch.equal(a.dstate, b.dstate)
    assert a.G.batches == b.G.batches and a.D.batches == b.D.batches and a.lam == b.lam
    for k in a.G.running:
        assert torch.equal(a.G.running[k], b.G.running[k]), k
    for k in a.D.running:
        assert torch.equal(a.D.running[k], b.D.running[k]), k
