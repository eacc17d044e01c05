"""The conv epilogue-statistics path at the benchmarked batch (B = 256) with canary words after every
buffer it writes ("what's weak" #2).

Round 2 recorded one illegal-address fault in the first eager conv round, under a rocprofv3 TA/TCP
counter pass, while the G-loss pass's discriminator forward ran its first ``groups = 1`` call of
``cgl_conv3x3_fwd_packed_stats`` + ``cgl_bn2d_fwd_stats`` (model/lsgan.py:76-91 on B images) on
partial / ticket buffers sized for the D step's 2B-image, ``groups = 2`` call.  These tests run every
statistics call of the round's geometry -- forward (D layers at n = 2B / groups 2 and n = B /
groups 1, G layers at 2B / groups 2 with the sliced finalize and its tickets) and backward
(``cgl_conv3x3_bwd_data_packed_stats`` + ``cgl_bn2d_bwd_stats``) -- on buffers followed by canary
words, twice in a row (the finalize tickets are monotonic), and require
  * every canary word unchanged (no write past st_part, the ticket scratch, y / dx),
  * the results equal to the plain two-pass BatchNorm2d (``bn2d_fwd`` / ``bn2d_bwd``) within fp32
    reduction-order tolerance.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"
CANARY = 4096                     # canary words after each buffer
PAT32 = 0x7FBADBAD                # a NaN bit pattern no kernel writes
PAT64 = 0x7FF0BADBADBADBAD


def ops():
    from cglgan import conv_ops
    return conv_ops


def padded(n, dtype=torch.float32):
    """A tensor of n elements followed by CANARY canary words (returns (view, whole buffer))."""
    if dtype == torch.float32:
        buf = torch.full((n + CANARY,), PAT32, dtype=torch.int32, device=DEV).view(torch.float32)
    elif dtype == torch.float64:
        buf = torch.full((n + CANARY,), PAT64, dtype=torch.int64, device=DEV).view(torch.float64)
    else:
        buf = torch.full((n + CANARY,), 0xA5, dtype=torch.uint8, device=DEV)
    return buf[:n], buf


def canary_ok(buf, n, what):
    tail = buf[n:]
    if buf.dtype == torch.float32:
        ok = bool((tail.view(torch.int32) == PAT32).all())
    elif buf.dtype == torch.float64:
        ok = bool((tail.view(torch.int64) == PAT64).all())
    else:
        ok = bool((tail == 0xA5).all())
    assert ok, f"{what}: canary words after the buffer were overwritten"


# (n images, input h = w, cin, cout, stride, up, groups): every statistics call of a B = 256 round
B = 256
FWD = [(2 * B, 32 // 2, 16, 32, 2, 0, 2), (B, 32 // 2, 16, 32, 2, 0, 1),      # D model.3 -> model.6
       (2 * B, 8, 32, 64, 2, 0, 2), (B, 8, 32, 64, 2, 0, 1),                 # D model.7 -> model.10
       (2 * B, 4, 64, 128, 2, 0, 2), (B, 4, 64, 128, 2, 0, 1),               # D model.11 -> model.14
       (2 * B, 8, 128, 128, 1, 1, 2), (2 * B, 16, 128, 64, 1, 1, 2)]         # G conv_blocks.1 / .5 (sliced)


@pytest.mark.parametrize("n,h,cin,cout,stride,up,groups", FWD)
def test_fwd_stats_canaries(n, h, cin, cout, stride, up, groups):
    O = ops()
    torch.manual_seed(n + h + cin + groups)
    ho = ((h << up) - 1) // stride + 1
    hw = ho * ho
    x = torch.randn(n, h, h, cin, device=DEV)
    w = torch.randn(cout, cin, 3, 3, device=DEV) * 0.1
    b = torch.randn(cout, device=DEV) * 0.1
    drop = (torch.rand(n, cout, device=DEV) > 0.25).float() / 0.75 if stride == 2 else None
    act = O.ACT_LEAKY if stride == 2 else O.ACT_NONE
    pk = O.PackSet()
    pk.add("x", "f", w, h, h, cin, cout, stride, up)
    pk.finalize(x.device).run()
    # the partial buffer sized for the largest (2B, groups 2) call of this layer, as ConvGanStep does
    nch = O.stat_chunks(2 * B if stride == 2 else n, h, h, cin, cout, stride, up, 2)
    assert nch > 0
    part, part_buf = padded(nch * cout * 2, torch.float64)
    scratch_n = int(O.bn2d_stats_scratch(cout, 2, x.device).numel())
    scratch, scratch_buf = padded(scratch_n, torch.uint8)
    scratch.zero_()
    y, y_buf = padded(n * hw * cout)
    y = y.view(n, ho, ho, cout)
    gam = 1 + 0.1 * torch.randn(cout, device=DEV)
    bet = 0.1 * torch.randn(cout, device=DEV)
    for rep in range(2):      # the sliced finalize's tickets are monotonic: run the pair twice
        O.conv3x3_fwd(x, None, b, y, n, h, h, cin, cout, stride, up, act=act, drop=drop, wp=pk["f"],
                      stats=(part, groups))
        out, out_buf = padded(n * hw * cout)
        rm, rv = torch.zeros(cout, device=DEV), torch.ones(cout, device=DEV)
        sm, si = torch.empty(groups, cout, device=DEV), torch.empty(groups, cout, device=DEV)
        O.bn2d_fwd_stats(part, y, n, hw, cout, gam, bet, out, groups=groups, running_mean=rm, running_var=rv,
                         act=O.ACT_NONE, save_mean=sm, save_invstd=si, scratch=scratch)
        # the plain two-pass BatchNorm on the same conv output
        ref = torch.empty(n * hw * cout, device=DEV)
        rm2, rv2 = torch.zeros(cout, device=DEV), torch.ones(cout, device=DEV)
        sm2, si2 = torch.empty(groups, cout, device=DEV), torch.empty(groups, cout, device=DEV)
        O.bn2d_fwd(y, n, hw, cout, gam, bet, ref, groups=groups, running_mean=rm2, running_var=rv2, train=True,
                   act=O.ACT_NONE, save_mean=sm2, save_invstd=si2)
        torch.cuda.synchronize()
        for t, bf, k in ((part, part_buf, "st_part"), (scratch, scratch_buf, "ticket scratch"),
                         (y.view(-1), y_buf, "conv output"), (out, out_buf, "bn output")):
            canary_ok(bf, t.numel(), f"{k} (rep {rep})")
        scale = float(ref.abs().max())
        assert float((out - ref).abs().max()) <= 2e-5 * scale, f"bn output vs two-pass (rep {rep})"
        assert torch.allclose(sm, sm2, rtol=1e-5, atol=1e-6) and torch.allclose(si, si2, rtol=1e-5, atol=1e-6)
        assert torch.allclose(rm, rm2, rtol=1e-5, atol=1e-6) and torch.allclose(rv, rv2, rtol=1e-5, atol=1e-6)


# input-gradient convs whose output feeds a BatchNorm backward: (n, conv input h, cin, cout, stride, up, groups)
BWD = [(2 * B, 8, 32, 64, 2, 0, 2), (B, 8, 32, 64, 2, 0, 1),          # dr[1] (model.6) from model.7's gradient
       (2 * B, 4, 64, 128, 2, 0, 2), (B, 4, 64, 128, 2, 0, 1),        # dr[2] (model.10) from model.11's gradient
       (B, 16, 128, 64, 1, 1, 1)]                                     # da1 (conv_blocks.2) from conv_blocks.5


@pytest.mark.parametrize("n,h,cin,cout,stride,up,groups", BWD)
def test_bwd_stats_canaries(n, h, cin, cout, stride, up, groups):
    O = ops()
    torch.manual_seed(7 * n + h + cin + groups)
    ho = ((h << up) - 1) // stride + 1
    hw_in = h * h
    w = torch.randn(cout, cin, 3, 3, device=DEV) * 0.1
    dy = torch.randn(n, ho, ho, cout, device=DEV)
    xbn = torch.randn(n, h, h, cin, device=DEV)                  # the BatchNorm input at dx's positions
    post = torch.randn(n, h, h, cin, device=DEV)                 # its post-activation (LeakyReLU' mask)
    pk = O.PackSet()
    pk.add("x", "b", w, h, h, cin, cout, stride, up, dir=1)
    pk.finalize(dy.device).run()
    nch = O.stat_chunks(n, h, h, cin, cout, stride, up, groups, bwd=True)
    assert nch > 0
    part, part_buf = padded(nch * cin * 2, torch.float64)
    sm = torch.randn(groups, cin, device=DEV) * 0.1
    si = 1 + 0.1 * torch.rand(groups, cin, device=DEV)
    gam = 1 + 0.1 * torch.randn(cin, device=DEV)
    for rep in range(2):
        dx, dx_buf = padded(n * hw_in * cin)
        dx = dx.view(n, h, h, cin)
        O.conv3x3_bwd_data(dy, None, dx, n, h, h, cin, cout, stride, up, wp=pk["b"],
                           stats=(part, groups, xbn, post, sm, 0.2))
        out, out_buf = padded(n * hw_in * cin)
        dg, db = torch.empty(cin, device=DEV), torch.empty(cin, device=DEV)
        O.bn2d_bwd_stats(part, dx, xbn, n, hw_in, cin, sm, si, gam, out, groups=groups, post=post, dgamma=dg, dbeta=db)
        ref = torch.empty(n * hw_in * cin, device=DEV)
        dg2, db2 = torch.empty(cin, device=DEV), torch.empty(cin, device=DEV)
        O.bn2d_bwd(dx, xbn, n, hw_in, cin, sm, si, gam, ref, groups=groups, post=post, dgamma=dg2, dbeta=db2)
        torch.cuda.synchronize()
        for t, bf, k in ((part, part_buf, "st_part"), (dx.view(-1), dx_buf, "dx"), (out, out_buf, "bn dx")):
            canary_ok(bf, t.numel(), f"{k} (rep {rep})")
        scale = float(ref.abs().max())
        assert float((out - ref).abs().max()) <= 5e-5 * scale, f"bn bwd vs two-pass (rep {rep})"
        assert torch.allclose(dg, dg2, rtol=5e-5, atol=1e-4) and torch.allclose(db, db2, rtol=5e-5, atol=1e-4)


@pytest.mark.parametrize("groups", [1, 2])
def test_bwd_n1_stats_bitwise(groups):
    """cgl_conv3x3_bwd_data_stats (the Conv2d(64, 1) input gradient with conv_blocks.6's backward partials per
    128-row chunk) + bn2d_bwd_stats(R = 128) against cgl_conv3x3_bwd_data + bn2d_bwd: bitwise equal (same
    chunks, rows, order), canaries intact, with post and with post_coef."""
    O = ops()
    torch.manual_seed(11 + groups)
    n, h, cin = 2 * 16, 32, 64
    hw = h * h
    w = torch.randn(1, cin, 3, 3, device=DEV) * 0.1
    dy = torch.randn(n, h, h, 1, device=DEV)
    xbn = torch.randn(n, h, h, cin, device=DEV)
    post = torch.randn(n, h, h, cin, device=DEV)
    sm = torch.randn(groups, cin, device=DEV) * 0.1
    si = 1 + 0.1 * torch.rand(groups, cin, device=DEV)
    gam = 1 + 0.1 * torch.randn(cin, device=DEV)
    coef = torch.randn(2 * cin, device=DEV)
    for pc in ([None, (coef, 0, 1)] if groups == 1 else [None]):
        kw = dict(post=None if pc else post, post_coef=pc) if pc else dict(post=post)
        part, part_buf = padded(n * hw // 128 * cin * 2, torch.float64)
        dx, dx_buf = padded(n * hw * cin)
        dx = dx.view(n, h, h, cin)
        O.conv3x3_bwd_data(dy, w, dx, n, h, h, cin, 1, 1, 0,
                           stats=(part, groups, xbn, kw.get("post"), sm, 0.2) + ((pc,) if pc else ()))
        out, out_buf = padded(n * hw * cin)
        dg, db = torch.empty(cin, device=DEV), torch.empty(cin, device=DEV)
        O.bn2d_bwd_stats(part, dx, xbn, n, hw, cin, sm, si, gam, out, groups=groups, dgamma=dg, dbeta=db, R=128, **kw)
        dx2 = torch.empty(n, h, h, cin, device=DEV)
        O.conv3x3_bwd_data(dy, w, dx2, n, h, h, cin, 1, 1, 0)
        ref = torch.empty(n * hw * cin, device=DEV)
        dg2, db2 = torch.empty(cin, device=DEV), torch.empty(cin, device=DEV)
        O.bn2d_bwd(dx2, xbn, n, hw, cin, sm, si, gam, ref, groups=groups, dgamma=dg2, dbeta=db2, **kw)
        torch.cuda.synchronize()
        for t, bf, k in ((part, part_buf, "st_part"), (dx.view(-1), dx_buf, "dx"), (out, out_buf, "bn dx")):
            canary_ok(bf, t.numel(), k)
        assert torch.equal(dx, dx2) and torch.equal(out, ref), pc is not None
        assert torch.equal(dg, dg2) and torch.equal(db, db2), pc is not None

