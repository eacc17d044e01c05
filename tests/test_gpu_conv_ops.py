"""Conv-path ops of libcglgan_hip (model/lsgan.py) vs a float64 torch-CPU reference of the same op.

Each op is called through the C ABI (cglgan.conv_ops) on NHWC device tensors and compared with
torch's own conv2d / interpolate / batch_norm / losses / autograd in float64 on the CPU.
Tolerance: fp32 result vs fp64 truth within 2e-5 relative to the output's max magnitude (the
MFMA accumulates exact fp32 products in k order; the phase-form upsampled convolutions add one
rounding of the combined weights).
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def ops():
    from cglgan import conv_ops
    return conv_ops


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


def close(got, ref, rel=2e-5, what=""):
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu()
    scale = max(float(ref.abs().max()), 1e-12)
    err = float((got - ref).abs().max())
    assert err <= rel * scale, f"{what}: max err {err:.3e} vs scale {scale:.3e}"


def _ref_conv(x, w, b, stride, up, act, slope, drop):
    if up:
        x = F.interpolate(x, scale_factor=2, mode="nearest")
    y = F.conv2d(x, w, b, stride, 1)
    if act == 1:
        y = F.leaky_relu(y, slope)
    elif act == 2:
        y = torch.tanh(y)
    if drop is not None:
        y = y * drop[:, :, None, None]
    return y


CONV_CASES = [
    # n, h, w, cin, cout, stride, up, act      (model/lsgan.py layer)
    (3, 8, 8, 128, 128, 1, 1, 0),     # G Upsample + Conv2d(128, 128)
    (2, 16, 16, 128, 64, 1, 1, 0),    # G Upsample + Conv2d(128, 64)
    (2, 32, 32, 64, 1, 1, 0, 2),      # G Conv2d(64, 1) + Tanh
    (3, 32, 32, 1, 16, 2, 0, 1),      # D Conv2d(1, 16, s2) + LeakyReLU (+ Dropout2d)
    (3, 16, 16, 16, 32, 2, 0, 1),     # D Conv2d(16, 32, s2)
    (2, 8, 8, 32, 64, 2, 0, 1),       # D Conv2d(32, 64, s2)
    (2, 4, 4, 64, 128, 2, 0, 1),      # D Conv2d(64, 128, s2)
    (2, 7, 7, 32, 64, 2, 0, 1),       # D on 28x28 inputs (odd sizes 7 -> 4)
    (2, 9, 7, 32, 48, 1, 0, 0),       # generic stride 1, ragged tiles
    (1, 5, 3, 16, 16, 1, 1, 1),       # ragged upsample
    (3, 7, 9, 64, 1, 1, 0, 2),        # one-output-channel conv, ragged (189 pixels: partial workgroups)
    (2, 20, 32, 64, 1, 1, 0, 2),      # tap-partial Conv2d(64, 1) with a partial 8-row tile
    # >= 2^28 MACs (no bias column): the LDS-staged weight gradient (cgl_conv_wgrad_lds)
    (16, 8, 8, 128, 128, 1, 1, 0),    # 128 x 128 workgroup tiles (WM = 2)
    (8, 16, 16, 128, 64, 1, 1, 0),    # 64 x 256 workgroup tiles (WM = 1)
    (32, 8, 8, 128, 128, 1, 0, 0),    # 9 direct taps, one tap per 128-column tile
]


@pytest.mark.parametrize("n,h,w,cin,cout,stride,up,act", CONV_CASES)
def test_conv3x3_fwd_bwd(n, h, w, cin, cout, stride, up, act):
    O = ops()
    g = torch.Generator().manual_seed(n * 1000 + h * 10 + cin + cout)
    x = torch.randn(n, cin, h, w, generator=g, dtype=torch.float64)
    wt = torch.randn(cout, cin, 3, 3, generator=g, dtype=torch.float64) / (3 * cin ** 0.5)
    b = torch.randn(cout, generator=g, dtype=torch.float64) * 0.1
    drop = None
    if act == 1:
        drop = (torch.rand(n, cout, generator=g) < 0.75).double() / 0.75
    ho, wo = O.conv_out_hw(h, w, stride, up)
    xd, wd, bd = nhwc(x).float().to(DEV), wt.float().to(DEV), b.float().to(DEV)
    dd = drop.float().to(DEV).contiguous() if drop is not None else None
    y = torch.empty(n, ho, wo, cout, device=DEV)
    O.conv3x3_fwd(xd, wd, bd, y, n, h, w, cin, cout, stride, up, act, 0.2, dd)
    xr = x.clone().requires_grad_(True)
    wr = wt.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    yr = _ref_conv(xr, wr, br, stride, up, act, 0.2, drop)
    close(nchw(y), yr, what="fwd")
    # backward of the convolution itself (pre-activation gradient dY)
    dy = torch.randn(n, cout, ho, wo, generator=g, dtype=torch.float64)
    x2 = x.clone().requires_grad_(True)
    w2 = wt.clone().requires_grad_(True)
    b2 = b.clone().requires_grad_(True)
    xin = F.interpolate(x2, scale_factor=2, mode="nearest") if up else x2
    F.conv2d(xin, w2, b2, stride, 1).backward(dy)
    dyd = nhwc(dy).float().to(DEV)
    dx = torch.empty(n, h, w, cin, device=DEV)
    O.conv3x3_bwd_data(dyd, wd, dx, n, h, w, cin, cout, stride, up)
    close(nchw(dx), x2.grad, what="bwd_data")
    dw = torch.empty(cout, cin, 3, 3, device=DEV)
    db = torch.empty(cout, device=DEV)
    O.conv3x3_bwd_weight(dyd, xd, dw, db, n, h, w, cin, cout, stride, up)
    close(dw, w2.grad, what="bwd_weight")
    close(db, b2.grad, what="bias grad")


@pytest.mark.parametrize("M,K,N,act", [(512, 100, 8192, 0), (64, 512, 1, 0), (512, 512, 1, 0), (7, 300, 1, 0),
                                       (37, 100, 70, 1), (16, 48, 33, 2)])
def test_dense(M, K, N, act):
    O = ops()
    g = torch.Generator().manual_seed(M + K + N)
    x = torch.randn(M, K, generator=g, dtype=torch.float64)
    w = torch.randn(N, K, generator=g, dtype=torch.float64) / K ** 0.5
    b = torch.randn(N, generator=g, dtype=torch.float64)
    y = torch.empty(M, N, device=DEV)
    O.dense_fwd(x.float().to(DEV), w.float().to(DEV), b.float().to(DEV), y, M, K, N, act, 0.2)
    ref = F.linear(x, w, b)
    ref = F.leaky_relu(ref, 0.2) if act == 1 else (torch.tanh(ref) if act == 2 else ref)
    close(y, ref, what="dense fwd")
    dy = torch.randn(M, N, generator=g, dtype=torch.float64)
    dx = torch.empty(M, K, device=DEV)
    O.dense_bwd_data(dy.float().to(DEV), w.float().to(DEV), dx, M, K, N)
    close(dx, dy @ w, what="dense bwd_data")
    dw = torch.empty(N, K, device=DEV)
    db = torch.empty(N, device=DEV)
    O.dense_bwd_weight(dy.float().to(DEV), x.float().to(DEV), dw, db, M, K, N)
    close(dw, dy.t() @ x, what="dense bwd_weight")
    close(db, dy.sum(0), what="dense bias grad")


@pytest.mark.parametrize("n,hw,C,groups,act", [(4, 256, 128, 2, 1), (6, 1024, 64, 2, 1), (3, 64, 32, 1, 0),
                                               (8, 4, 128, 2, 0), (2, 16, 64, 1, 1)])
def test_bn2d_fwd_bwd(n, hw, C, groups, act):
    O = ops()
    g = torch.Generator().manual_seed(n + hw + C)
    x = torch.randn(n, hw, C, generator=g, dtype=torch.float64) * 2 + 0.5
    gam = 1 + 0.1 * torch.randn(C, generator=g, dtype=torch.float64)
    bet = 0.1 * torch.randn(C, generator=g, dtype=torch.float64)
    rm0 = 0.1 * torch.randn(C, generator=g, dtype=torch.float64)
    rv0 = 1 + 0.1 * torch.rand(C, generator=g, dtype=torch.float64)
    xd = x.float().to(DEV)
    gd, bd = gam.float().to(DEV), bet.float().to(DEV)
    rm, rv = rm0.float().to(DEV), rv0.float().to(DEV)
    y = torch.empty_like(xd)
    sm = torch.empty(groups, C, device=DEV)
    si = torch.empty(groups, C, device=DEV)
    O.bn2d_fwd(xd, n, hw, C, gd, bd, y, groups=groups, eps=0.8, momentum=0.1, running_mean=rm, running_var=rv,
               train=True, act=act, save_mean=sm, save_invstd=si)
    # reference: one F.batch_norm call per group, in order (the reference's separate forward calls)
    ng = n // groups
    rmr, rvr = rm0.clone(), rv0.clone()
    outs, xs = [], []
    for q in range(groups):
        xq = x[q * ng:(q + 1) * ng].permute(0, 2, 1).reshape(ng, C, hw, 1).clone().requires_grad_(True)
        o = F.batch_norm(xq, rmr, rvr, gam, bet, True, 0.1, 0.8)
        if act:
            o = F.leaky_relu(o, 0.2)
        outs.append(o)
        xs.append(xq)
    yr = torch.cat([o.reshape(ng, C, hw).permute(0, 2, 1) for o in outs])
    close(y.view(n, hw, C), yr, what="bn fwd")
    close(rm, rmr, what="running_mean")
    close(rv, rvr, what="running_var")
    dy = torch.randn(n, hw, C, generator=g, dtype=torch.float64)
    for q, o in enumerate(outs):
        o.backward(dy[q * ng:(q + 1) * ng].permute(0, 2, 1).reshape(ng, C, hw, 1))
    dxr = torch.cat([xq.grad.reshape(ng, C, hw).permute(0, 2, 1) for xq in xs])
    dx = torch.empty_like(xd)
    dgam = torch.empty(C, device=DEV)
    dbet = torch.empty(C, device=DEV)
    O.bn2d_bwd(dy.float().to(DEV), xd, n, hw, C, sm, si, gd, dx, groups=groups, post=y if act else None,
               dgamma=dgam, dbeta=dbet)
    close(dx, dxr, rel=5e-5, what="bn bwd")
    # gamma / beta grads of the summed groups
    gref = torch.zeros(C, dtype=torch.float64)
    bref = torch.zeros(C, dtype=torch.float64)
    for q in range(groups):
        xq = x[q * ng:(q + 1) * ng].permute(0, 2, 1).reshape(ng, C, hw, 1)
        gq = gam.clone().requires_grad_(True)
        bq = bet.clone().requires_grad_(True)
        o = F.batch_norm(xq, None, None, gq, bq, True, 0.1, 0.8)
        if act:
            o = F.leaky_relu(o, 0.2)
        o.backward(dy[q * ng:(q + 1) * ng].permute(0, 2, 1).reshape(ng, C, hw, 1))
        gref += gq.grad
        bref += bq.grad
    close(dgam, gref, rel=5e-5, what="dgamma")
    close(dbet, bref, rel=5e-5, what="dbeta")


def test_bn2d_eval_and_fused_dropout_leaky_bwd():
    """Eval mode uses running stats; backward with post_out/drop = Conv->LReLU->Dropout2d->BN block."""
    O = ops()
    g = torch.Generator().manual_seed(7)
    n, hw, C = 4, 16, 64
    q = F.leaky_relu(torch.randn(n, hw, C, generator=g, dtype=torch.float64), 0.2)
    drop = (torch.rand(n, C, generator=g) < 0.75).double() / 0.75
    q = q * drop[:, None, :]
    gam = 1 + 0.1 * torch.randn(C, generator=g, dtype=torch.float64)
    bet = 0.1 * torch.randn(C, generator=g, dtype=torch.float64)
    rm = 0.1 * torch.randn(C, generator=g, dtype=torch.float64)
    rv = 1 + 0.1 * torch.rand(C, generator=g, dtype=torch.float64)
    y = torch.empty(n, hw, C, device=DEV)
    O.bn2d_fwd(q.float().to(DEV), n, hw, C, gam.float().to(DEV), bet.float().to(DEV), y, running_mean=rm.float().to(DEV),
               running_var=rv.float().to(DEV), train=False)
    ref = F.batch_norm(q.permute(0, 2, 1), rm, rv, gam, bet, False, 0.1, 0.8).permute(0, 2, 1)
    close(y, ref, what="bn eval")
    # backward through BN (train) then Dropout2d + LeakyReLU, vs autograd from the conv output c
    c = torch.randn(n, hw, C, generator=g, dtype=torch.float64).requires_grad_(True)
    qq = F.leaky_relu(c, 0.2) * drop[:, None, :]
    o = F.batch_norm(qq.permute(0, 2, 1), None, None, gam, bet, True, 0.1, 0.8).permute(0, 2, 1)
    dy = torch.randn(n, hw, C, generator=g, dtype=torch.float64)
    o.backward(dy)
    qd = qq.detach().float().to(DEV)
    yd = torch.empty_like(qd)
    sm = torch.empty(1, C, device=DEV)
    si = torch.empty(1, C, device=DEV)
    O.bn2d_fwd(qd, n, hw, C, gam.float().to(DEV), bet.float().to(DEV), yd, save_mean=sm, save_invstd=si)
    dc = torch.empty_like(qd)
    O.bn2d_bwd(dy.float().to(DEV), qd, n, hw, C, sm, si, gam.float().to(DEV), dc, post_out=qd,
               drop=drop.float().to(DEV).contiguous())
    close(dc, c.grad, rel=5e-5, what="bn+dropout+leaky bwd")
    # the standalone Dropout2d + LeakyReLU backward (block 1 of D has no BatchNorm)
    dq = torch.randn(n, hw, C, generator=g, dtype=torch.float64)
    c2 = c.detach().clone().requires_grad_(True)
    (F.leaky_relu(c2, 0.2) * drop[:, None, :]).backward(dq)
    out = torch.empty_like(qd)
    O.act_drop_bwd(dq.float().to(DEV), qd, drop.float().to(DEV).contiguous(), n, hw, C, out)
    close(out, c2.grad, what="dropout+leaky bwd")


@pytest.mark.parametrize("kind,C", [("mse", 1), ("bce", 1), ("bce_prob", 1), ("ce", 2)])
@pytest.mark.parametrize("target", [0, 1])
def test_adv_loss(kind, C, target):
    O = ops()
    g = torch.Generator().manual_seed(3)
    M = 300
    x = torch.randn(M, C, generator=g, dtype=torch.float64)
    if kind == "bce_prob":
        x = torch.sigmoid(x)
    xr = x.clone().requires_grad_(True)
    if kind == "mse":
        l = F.mse_loss(xr, torch.full_like(xr, float(target)))
    elif kind == "bce":
        l = F.binary_cross_entropy(torch.sigmoid(xr), torch.full_like(xr, float(target)))
    elif kind == "bce_prob":
        l = F.binary_cross_entropy(xr, torch.full_like(xr, float(target)))
    else:
        l = F.cross_entropy(xr, torch.full((M,), target, dtype=torch.long))
    (0.5 * l).backward()
    lo = torch.empty(1, device=DEV)
    gr = torch.empty(M, C, device=DEV)
    O.adv_loss(x.float().to(DEV), M, C, kind, target, 0.5, lo, gr)
    close(lo, l.detach().view(1), rel=1e-6, what="loss")
    close(gr, xr.grad, rel=1e-5, what="loss grad")


def test_dropout_mask_statistics():
    O = ops()
    m = torch.empty(512, 128, device=DEV)
    O.dropout2d_mask(m, 512, 128, 0.25, 1234, 7)
    u = torch.unique(m.cpu())
    assert set(float(v) for v in u) <= {0.0, float(torch.tensor(1.0) / torch.tensor(0.75))}
    keep = float((m > 0).float().mean())
    assert abs(keep - 0.75) < 0.01
    m2 = torch.empty_like(m)
    O.dropout2d_mask(m2, 512, 128, 0.25, 1234, 7)
    assert torch.equal(m, m2)
    O.dropout2d_mask(m2, 512, 128, 0.25, 1234, 8)
    assert not torch.equal(m, m2)


def test_layout_and_gather():
    O = ops()
    x = torch.randn(3, 128, 64, device=DEV)
    y = torch.empty(3, 64, 128, device=DEV)
    O.nchw_to_nhwc(x, y, 3, 128, 64)
    assert torch.equal(y, x.permute(0, 2, 1))
    z = torch.empty_like(x)
    O.nhwc_to_nchw(y, z, 3, 128, 64)
    assert torch.equal(z, x)
    src = torch.randn(50, 1024, device=DEV)
    idx = torch.tensor([3, 49, 0, 7], dtype=torch.int32, device=DEV)
    dst = torch.empty(4, 1024, device=DEV)
    O.gather_rows(src, idx, 0, 4, 1024, dst)
    assert torch.equal(dst, src[idx.long()])
    O.gather_rows(src, None, 10, 4, 1024, dst)
    assert torch.equal(dst, src[10:14])


@pytest.mark.parametrize("M", [16, 512])
def test_linear_gather_nhwc(M):
    """cgl_linear_prepare_gather with the conv round's NCHW -> NHWC feature permutation (model/lsgan.py:23-25):
    bit for bit the plain prepared Linear's output transposed to NHWC, and close to the fp64 torch Linear;
    the bias packed in that order by the 1x1 input-gradient pack (PackSet dir 1) is its exact transpose.
    cgl_linear_prepare_wgrad_nhwc: the weight / bias gradient of the same Linear from an NHWC gradient."""
    O = ops()
    g = torch.Generator(device=DEV).manual_seed(11)
    x = torch.randn(M, 100, device=DEV, generator=g)
    w = torch.randn(8192, 100, device=DEV, generator=g) * 0.1
    b = torch.randn(8192, device=DEV, generator=g)
    ps = O.PackSet()
    ps.add("G", "l1b", b, 1, 1, 64, 128, 1, 0, ks=1, dir=1)
    ps = ps.finalize(torch.device(DEV))
    ps.run()
    n = torch.arange(8192, dtype=torch.int32, device=DEV)
    rows = ((n % 128) * 64 + n // 128).to(torch.int32).contiguous()
    y0 = torch.empty(M, 8192, device=DEV)
    y1 = torch.empty(M, 8, 8, 128, device=DEV)
    O.PreparedLinear(0, x, w, b, y0, None, M, 8192, 100)()
    O.PreparedLinear(0, x, w, ps["l1b"], y1, None, M, 8192, 100, b_rows=rows)()
    torch.cuda.synchronize()
    assert torch.equal(ps["l1b"].view(64, 128), b.view(128, 64).t())
    assert torch.equal(y1, y0.view(M, 128, 8, 8).permute(0, 2, 3, 1))
    ref = (x.double() @ w.double().t() + b.double()).view(M, 128, 8, 8).permute(0, 2, 3, 1)
    assert (y1.double() - ref).abs().max() <= 2e-5 * ref.abs().max()
    with pytest.raises(ValueError):
        O.PreparedLinear(0, x, w, b, y1, None, M, 8192, 100, b_rows=rows + 8192)
    # a table of no shift form goes through the per-launch index load: bitwise the Linear on the gathered W
    rnd = torch.randperm(8192, device=DEV, generator=g).to(torch.int32)
    y2, y3 = torch.empty(M, 8192, device=DEV), torch.empty(M, 8192, device=DEV)
    O.PreparedLinear(0, x, w, b, y2, None, M, 8192, 100, b_rows=rnd)()
    O.PreparedLinear(0, x, w[rnd.long()].contiguous(), b, y3, None, M, 8192, 100)()
    torch.cuda.synchronize()
    assert torch.equal(y2, y3)
    # the weight + bias gradient from the NHWC gradient (cgl_linear_prepare_wgrad_nhwc): bit for bit op 2 on
    # the NCHW transpose, close to fp64
    dy = torch.randn(M, 8, 8, 128, device=DEV, generator=g)
    dyc = dy.permute(0, 3, 1, 2).contiguous().view(M, 8192)
    dw0, db0 = torch.empty(8192, 100, device=DEV), torch.empty(8192, device=DEV)
    dw1, db1 = torch.full((8192, 100), float("nan"), device=DEV), torch.full((8192,), float("nan"), device=DEV)
    O.PreparedLinear(2, dyc, x, None, dw0, db0, M, 8192, 100)()
    O.PreparedLinear(2, dy, x, None, dw1, db1, M, 8192, 100, nhwc=(128, 64))()
    torch.cuda.synchronize()
    assert torch.equal(dw1, dw0) and torch.equal(db1, db0)
    rw = dyc.double().t() @ x.double()
    assert (dw1.double() - rw).abs().max() <= 2e-5 * rw.abs().max()
    assert (db1.double() - dyc.double().sum(0)).abs().max() <= 2e-5 * dyc.double().sum(0).abs().max()
    with pytest.raises(ValueError):
        O.PreparedLinear(2, dy, x, None, dw1, db1, M, 8192, 100, nhwc=(128, 32))


def test_adam_multi_matches_torch_single_tensor():
    O = ops()
    from oracle.gan_oracle import Adam
    g = torch.Generator().manual_seed(5)
    shapes = [(33, 7), (8192,), (1,), (300, 3)]
    ps = [torch.randn(*s, generator=g) for s in shapes]
    ref = [p.clone().requires_grad_(True) for p in ps]
    opt = Adam(ref)
    dp = [p.to(DEV) for p in ps]
    dm = [torch.zeros_like(p) for p in dp]
    dv = [torch.zeros_like(p) for p in dp]
    for step in range(1, 4):
        grads = [torch.randn(*s, generator=g) for s in shapes]
        for r, gr in zip(ref, grads):
            r.grad = gr.clone()
        opt.step()
        O.adam_multi(dp, [gr.to(DEV) for gr in grads], dm, dv, step)
    # torch's CPU op order; GPU sqrt / division may differ by an ulp (same bound as test_gpu_ops.py)
    for a, b, m, mr, v, vr in zip(dp, ref, dm, opt.m, dv, opt.v):
        close(a, b, rel=1e-6, what="param")
        close(m, mr, rel=1e-6, what="exp_avg")
        close(v, vr, rel=1e-6, what="exp_avg_sq")


@pytest.mark.parametrize("n", [1, 8, 512])
def test_dense1_head_nhwc_bitwise(n):
    """D head of model/lsgan.py:96-97 (out.view(B, -1) -> Linear(512, 1)) from the NHWC 2x2x128 map:
    cgl_dense1_fwd_nhwc equals nhwc_to_nchw + dense_fwd(N=1) bit for bit (and writes the same view),
    cgl_dense1_bwd_data_nhwc equals dense_bwd_data(K=1) + nchw_to_nhwc bit for bit, both close to fp64."""
    O = ops()
    g = torch.Generator(device="cpu").manual_seed(n)
    x = torch.randn(n, 2, 2, 128, generator=g).to(DEV)
    w = (torch.randn(1, 512, generator=g) * 0.05).to(DEV)
    b = torch.randn(1, generator=g).to(DEV)
    dy = torch.randn(n, 1, generator=g).to(DEV)
    flat = torch.empty(n, 512, device=DEV)
    y_old = torch.empty(n, 1, device=DEV)
    O.nhwc_to_nchw(x, flat, n, 128, 4)
    O.dense_fwd(flat, w, b, y_old, n, 512, 1)
    y_new, flat_new = torch.empty(n, 1, device=DEV), torch.full((n, 512), float("nan"), device=DEV)
    O.dense1_fwd_nhwc(x, w, b, y_new, n, 128, 4, flat=flat_new)
    y_noflat = torch.empty(n, 1, device=DEV)
    O.dense1_fwd_nhwc(x, w, b, y_noflat, n, 128, 4)
    dflat, dx_old = torch.empty(n, 512, device=DEV), torch.empty(n, 2, 2, 128, device=DEV)
    O.dense_bwd_data(dy, w, dflat, n, 512, 1)
    O.nchw_to_nhwc(dflat, dx_old, n, 128, 4)
    dx_new = torch.empty(n, 2, 2, 128, device=DEV)
    O.dense1_bwd_data_nhwc(dy, w, dx_new, n, 128, 4)
    torch.cuda.synchronize()
    assert torch.equal(y_new, y_old) and torch.equal(y_noflat, y_old)
    assert torch.equal(flat_new, flat)
    assert torch.equal(dx_new, dx_old)
    xr = nchw(x.cpu().double()).reshape(n, 512)
    close(y_new, xr @ w.cpu().double().t() + b.cpu().double(), what="head fwd")
    close(dx_new, nhwc((dy.cpu().double() @ w.cpu().double()).reshape(n, 128, 2, 2)), what="head bwd")
