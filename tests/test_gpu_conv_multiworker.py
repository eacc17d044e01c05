"""N conv-GAN workers (model/lsgan.py) on one GPU in lockstep (cglgan.exchange.ConvLocalComm, the
same phase A / gather / alpha / sum / phase B sequence ConvWorkerExchange runs over RCCL) vs
oracle/conv_oracle.ConvCapgan, in which the reference's Server backpropagates
F_max = sum alpha_i l_i - 0.001 lambda through every worker's D (capgan.py:211-262, data-size weights
beta) or F = mean l (MDGAN/MNIST/mdgan.py:203-205).  Tolerance rule of test_gpu_conv_step:
||hip - fp64|| <= max(1e-5 ||fp64||, 4 ||fp32 - fp64||).  Also: the replicated G stays bitwise
identical on every worker.
"""
import pytest
import torch

from oracle import conv_oracle as CO

pytestmark = pytest.mark.gpu
PRE_BN_BIAS = {"conv_blocks.1.bias", "conv_blocks.5.bias"}


def _err(a, b):
    return float((a.detach().double().cpu() - b.detach().double().cpu()).norm())


def _check(name, hip, o64, o32, fails, tol=1e-5):
    e = _err(hip, o64)
    bound = max(tol * float(o64.detach().double().norm()), 4 * _err(o32, o64), 1e-12)
    if e > bound:
        fails.append(f"{name}: err {e:.3e} > bound {bound:.3e}")


def _split(sd):
    return ({k: v.cpu() for k, v in sd.items() if "running" not in k and "num_batches" not in k},
            {k: v.cpu() for k, v in sd.items() if "running" in k or "num_batches" in k})


@pytest.mark.parametrize("weighting,beta", [("capgan", [0.25, 0.75]), ("mean", [0.5, 0.5])])
def test_conv_two_workers(weighting, beta):
    from cglgan.conv_step import ConvGanStep
    from cglgan.exchange import ConvLocalComm
    torch.set_num_threads(4)
    N, B = 2, 8
    steps = []
    for r in range(N):
        s = ConvGanStep(B, loss="mse", seed=7, n_workers=N, rank=r, weighting=weighting)
        s.init_default(20211212, 20211213 + r)
        s.beta = list(beta)
        steps.append(s)
    gp, gb = _split(steps[0].G.state_dict())
    ds = [_split(s.D.state_dict()) for s in steps]
    o64 = CO.ConvCapgan(gp, gb, [d[0] for d in ds], [d[1] for d in ds], beta, weighting=weighting,
                        dtype=torch.float64)
    o32 = CO.ConvCapgan(gp, gb, [d[0] for d in ds], [d[1] for d in ds], beta, weighting=weighting,
                        dtype=torch.float32)
    comm = ConvLocalComm(steps)
    g = torch.Generator().manual_seed(9)
    for rnd in range(2):
        reals = [torch.rand(B, 1, 32, 32, generator=g) * 2 - 1 for _ in range(N)]
        comm.round(rnd, reals=[x.cuda() for x in reals])
        torch.cuda.synchronize()
        z = steps[0].z.cpu()
        masks = [([m[:B].cpu() for m in s.mask_d], [m[B:].cpu() for m in s.mask_d], [m.cpu() for m in s.mask_g])
                 for s in steps]
        r64 = o64.round(z[:B], z[B:], reals, masks)
        r32 = o32.round(z[:B], z[B:], reals, masks)
        fails = []
        hip_l = torch.stack([s.lbuf[2].cpu() for s in steps])
        _check("losses", hip_l, r64["losses"], r32["losses"], fails)
        _check("Xg", steps[0].xg().permute(0, 3, 1, 2), r64["Xg"], r32["Xg"], fails)
        for k, v in r64["g_grads"].items():
            if k not in PRE_BN_BIAS:
                _check(f"r{rnd} G grad {k}", steps[0].G.grads[k], v, r32["g_grads"][k], fails)
        for i, s in enumerate(steps):
            for k, v in r64["d_grads"][i].items():
                _check(f"r{rnd} D{i} grad {k}", s.D.grads[k], v, r32["d_grads"][i][k], fails)
            for k, v in s.D.params.items():
                _check(f"r{rnd} D{i} param {k}", v, o64.dps[i][k], o32.dps[i][k], fails)
        for k, v in steps[0].G.params.items():
            if k not in PRE_BN_BIAS:
                _check(f"r{rnd} G param {k}", v, o64.gp[k], o32.gp[k], fails)
        assert not fails, "\n".join(fails)
        assert torch.equal(steps[0].G.p, steps[1].G.p), "replicated G diverged"
        assert abs(steps[0].lam - o64.lam) <= 1e-12
