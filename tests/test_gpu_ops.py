"""Single HIP ops vs plain PyTorch fp32 on the GPU (the kernels under the fused step).

Tolerance: fp32 MFMA is an exact k-ordered fma chain; only the summation order differs from
torch's GEMM, so <= 1e-5 relative (norm) is required.
"""
import ctypes

import pytest
import torch

from cglgan import _lib as C

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _rel(a, b):
    return float((a.double() - b.double()).norm() / max(b.double().norm(), 1e-30))


def _ws():
    return torch.zeros(C.lib.cgl_op_workspace_bytes(), dtype=torch.uint8, device="cuda")


def _s():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


SHAPES = [(256, 128, 100), (512, 784, 1024), (37, 50, 100), (1, 2, 256), (300, 33, 2), (64, 1, 32), (512, 1024, 512)]


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("act", [0, 1, 2])
def test_linear_fwd(M, N, K, act):
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N + K)
    X = torch.randn(M, K, device="cuda", generator=g)
    W = torch.randn(N, K, device="cuda", generator=g) * 0.05
    b = torch.randn(N, device="cuda", generator=g)
    Y = torch.empty(M, N, device="cuda")
    ws = _ws()
    C.check(C.lib.cgl_linear_fwd(_p(X), _p(W), _p(b), _p(Y), M, N, K, act, 0.2, _p(ws), ws.numel(), _s()))
    ref = torch.nn.functional.linear(X, W, b)
    ref = [ref, torch.nn.functional.leaky_relu(ref, 0.2), torch.tanh(ref)][act]
    assert _rel(Y, ref) <= TOL


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_linear_bwd(M, N, K):
    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + K)
    X = torch.randn(M, K, device="cuda", generator=g)
    W = torch.randn(N, K, device="cuda", generator=g) * 0.05
    dY = torch.randn(M, N, device="cuda", generator=g)
    dX = torch.empty(M, K, device="cuda")
    dW = torch.empty(N, K, device="cuda")
    db = torch.empty(N, device="cuda")
    ws = _ws()
    C.check(C.lib.cgl_linear_bwd_data(_p(dY), _p(W), _p(dX), M, N, K, _p(ws), ws.numel(), _s()))
    C.check(C.lib.cgl_linear_bwd_weight(_p(dY), _p(X), _p(dW), _p(db), M, N, K, _p(ws), ws.numel(), _s()))
    assert _rel(dX, dY @ W) <= TOL
    assert _rel(dW, dY.t() @ X) <= TOL
    assert _rel(db, dY.sum(0)) <= TOL


def test_adam_matches_torch_single_tensor():
    from oracle.gan_oracle import Adam
    n = 100003
    g = torch.Generator().manual_seed(1)
    p0 = torch.randn(n, generator=g)
    ref_p = p0.clone().requires_grad_(True)
    opt = Adam([ref_p])
    p, m, v = p0.cuda(), torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
    ws = _ws()
    for t in range(1, 6):
        grad = torch.randn(n, generator=g)
        ref_p.grad = grad.clone()
        opt.step()
        gd = grad.cuda()
        C.check(C.lib.cgl_adam_step(_p(p), _p(gd), _p(m), _p(v), n, t, 2e-4, 0.5, 0.999, 1e-8, _p(ws), ws.numel(),
                                    _s()))
    torch.cuda.synchronize()
    assert _rel(p.cpu(), ref_p.detach()) <= 1e-6
    assert _rel(m.cpu(), opt.m[0]) <= 1e-6
    assert _rel(v.cpu(), opt.v[0]) <= 1e-6


def test_normal_fill_moments():
    n = 1 << 20
    out = torch.empty(n, device="cuda")
    C.check(C.lib.cgl_normal_fill(_p(out), n, 1234, 0, 0, _s()))
    torch.cuda.synchronize()
    assert abs(out.mean().item()) < 5e-3
    assert abs(out.std().item() - 1.0) < 5e-3
    out2 = torch.empty(n, device="cuda")
    C.check(C.lib.cgl_normal_fill(_p(out2), n, 1234, 0, 0, _s()))
    torch.cuda.synchronize()
    assert torch.equal(out, out2)
