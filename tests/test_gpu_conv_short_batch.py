"""The short final batch on the conv path (DataLoader(shuffle=True) without drop_last, capgan.py:282,326-331):
a shard of n rows gives ceil(n / B) batches per pass, the last one of n mod B rows, and the reference's D step
runs its real call on that short batch -- BatchNorm2d statistics over its images only, the loss a mean over
them.  The fused conv round keeps its launch geometry (B images per call) and carries the real call's image
count on the device (ConvGanStep.nv): the padding images are left out of the real call's statistics, loss and
gradients (cglgan.conv_ops nvalid).

* one round with an explicit short real batch vs the conv oracle fed the same short batch (fp64 / fp32, the
  tolerance of tests/test_gpu_conv_step.py, the oracle following the GPU's LeakyReLU branches);
* the device and host samplers: each pass covers every row of a non-multiple shard exactly once, the pass's
  last batch short, and nv matches;
* a free-running trajectory across a pass boundary (non-multiple shard, the round's own sampler) vs the fp64
  oracle fed the sampled rows: losses within 1e-4."""
import pytest
import torch

from oracle import conv_oracle as CO
from test_gpu_conv_step import PRE_BN_BIAS, SUM_BIASES, _check, _check_signs, _check_sum, _gpu_signs

pytestmark = pytest.mark.gpu


def _oracles(st):
    gp0, dp0 = st.G.state_dict(), st.D.state_dict()
    split = lambda sd: ({k: v.cpu() for k, v in sd.items() if "running" not in k and "num_batches" not in k},
                        {k: v.cpu() for k, v in sd.items() if "running" in k or "num_batches" in k})
    gp, gb = split(gp0)
    dp, db = split(dp0)
    return (CO.ConvGan(gp, gb, dp, db, loss=st.loss, dtype=torch.float64),
            CO.ConvGan(gp, gb, dp, db, loss=st.loss, dtype=torch.float32))


def _recording(st):
    d_calls = []
    fwd = st._d_forward

    def rec(x, n, groups, masks, **kw):
        fwd(x, n, groups, masks, **kw)
        d_calls.append([q[:n].clone() for q in st.q])
    st._d_forward = rec
    return d_calls


@pytest.mark.parametrize("B,nr,loss", [(8, 5, "mse"), (8, 3, "bce"), (256, 96, "mse")])
def test_short_real_call_vs_oracle(B, nr, loss):
    """(256, 96): the bench's shard of 60,000 rows ends every pass with a batch of 96."""
    from cglgan.conv_step import ConvGanStep
    torch.set_num_threads(4)
    st = ConvGanStep(B, loss=loss, seed=3)
    st.init_default(20211212, 20211213)
    o64, o32 = _oracles(st)
    d_calls = _recording(st)
    real = torch.rand(nr, 1, 32, 32, generator=torch.Generator().manual_seed(9)) * 2 - 1
    st.run(real=real.cuda())
    torch.cuda.synchronize()
    assert int(st.nv.item()) == nr
    z = st.z.cpu()
    mr = [m[:nr].cpu() for m in st.mask_d]
    mf = [m[B:].cpu() for m in st.mask_d]
    mg = [m.cpu() for m in st.mask_g]
    signs, valid = _gpu_signs(st, d_calls)
    signs["dr"] = [m[:nr] for m in signs["dr"]]
    valid["dr"] = [m[:nr] for m in valid["dr"]]
    trace = {}
    r64 = o64.round(z[:B], z[B:], real, mr, mf, mg, signs=signs, trace=trace)
    r32 = o32.round(z[:B], z[B:], real, mr, mf, mg, signs=signs)
    _check_signs(signs, valid, trace)
    s, gg, dg = st.stats(), st.G.grads, st.D.grads
    fails = []
    for k in ("d_real", "d_fake", "g_loss"):
        _check(k, torch.tensor(s[k]), torch.tensor(r64[k]), torch.tensor(r32[k]), fails)
    for k, v in r64["d_grads"].items():
        _check("D grad " + k, dg[k], v, r32["d_grads"][k], fails)
    for k, v in r64["g_grads"].items():
        if k in PRE_BN_BIAS:
            continue
        if k in SUM_BIASES:
            _check_sum("G grad " + k, gg[k], v, r32["g_grads"][k], st.dc3g, fails)
        else:
            _check("G grad " + k, gg[k], v, r32["g_grads"][k], fails)
    for k, v in st.D.params.items():
        _check("D param " + k, v, o64.dp[k], o32.dp[k], fails)
    for k, v in st.D.running.items():          # running statistics over the short call's images only
        _check("D " + k, v, o64.db[k], o32.db[k], fails)
    assert not fails, "\n".join(fails)


@pytest.mark.parametrize("graph", [False, True])
def test_sampler_passes_cover_the_shard(graph):
    from cglgan.conv_step import ConvGanStep
    B, n = 8, 27                                  # 3 full batches + one of 3 per pass
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        data = torch.arange(n, dtype=torch.float32, device="cuda")[:, None].repeat(1, 1024) / n
        st = ConvGanStep(B, seed=13, data=data, graph=graph)
        st.init_default(1, 2)
        seen, nvs = [], []
        for _ in range(9):
            st.run()
            torch.cuda.synchronize()
            nv = int(st.nv.item())
            nvs.append(nv)
            seen.append([int(round(float(v) * n)) for v in st.x3[:nv, 0, 0, 0].cpu()])
    # eager: the host sampler, batches 0.. of the stream; graph: round 0 eager (host sampler), then the device
    # sampler with batch index = round (rounds 4..7 = one whole pass of 4 batches)
    passes = [range(0, 4), range(4, 8)] if not graph else [range(4, 8)]
    for p in passes:
        rows = sum((seen[r] for r in p), [])
        assert sorted(rows) == list(range(n)), (p, rows)
        assert [nvs[r] for r in p] == [8, 8, 8, 3], nvs


def test_trajectory_across_pass_boundary():
    """B = 8 over a shard of 20 rows (passes of 8, 8, 4), 6 rounds eager: each round's losses vs the fp64 oracle
    fed the rows the round sampled (read back), Dropout2d scales injected; free-running (1e-4)."""
    from cglgan.conv_step import ConvGanStep
    torch.set_num_threads(4)
    B, n = 8, 20
    data = (torch.rand(n, 1024, generator=torch.Generator().manual_seed(4)) * 2 - 1).cuda()
    st = ConvGanStep(B, loss="mse", seed=5, data=data)
    st.init_default(20211212, 20211213)
    o64, o32 = _oracles(st)
    short = 0
    for r in range(6):
        st.run()
        torch.cuda.synchronize()
        nv = int(st.nv.item())
        short += nv < B
        real = st.x3[:nv].permute(0, 3, 1, 2).cpu()
        z = st.z.cpu()
        mr = [m[:nv].cpu() for m in st.mask_d]
        mf = [m[B:].cpu() for m in st.mask_d]
        mg = [m.cpu() for m in st.mask_g]
        r64 = o64.round(z[:B], z[B:], real, mr, mf, mg)
        r32 = o32.round(z[:B], z[B:], real, mr, mf, mg)
        s = st.stats()
        for k in ("d_real", "d_fake", "g_loss"):
            ref = r64[k]
            assert abs(s[k] - ref) <= max(1e-4 * abs(ref), 4 * abs(r32[k] - ref)), (r, k, s[k], ref)
    assert short == 2                               # rounds 2 and 5 ran short batches of 4
