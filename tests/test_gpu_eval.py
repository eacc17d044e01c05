"""cgl_kl_score (cglgan.evaluation.kl_score) vs numpy / scipy, the calls CGLGAN/2DMG/main.py:63-101
makes: integer histograms bit-exact against np.histogram2d (edge rules included: points on the upper
edge, outside the range, NaN); the score within 1e-12 relative of scipy.stats.entropy (device log vs
libm)."""
import numpy as np
import pytest
import torch
from scipy.stats import entropy

pytestmark = pytest.mark.gpu


def _ref(real, gen, bins=16):
    cr, _, _ = np.histogram2d(real[:, 0], real[:, 1], bins=bins, range=[[-1, 1], [-1, 1]])
    cg, _, _ = np.histogram2d(gen[:, 0], gen[:, 1], bins=bins, range=[[-1, 1], [-1, 1]])
    r, g = [], []
    for i in range(len(cr)):
        for j in range(len(cr)):
            if cr[i][j] != 0:
                r.append(cr[i][j])
                g.append(cg[i][j])
    return cr, cg, entropy(g, r)


def _ring(n, g, std=0.01):
    th = np.linspace(0, 2 * (1 - 1 / 8) * np.pi, 8)
    c = g.integers(0, 8, n)
    return (np.stack([np.sin(th[c]), np.cos(th[c])], 1) + std * g.standard_normal((n, 2))).astype(np.float32)


def test_kl_score_matches_numpy_scipy():
    from cglgan.evaluation import kl_score
    g = np.random.default_rng(0)
    real = _ring(10000, g)
    gen = _ring(2000, g, std=0.05)
    gen[:5] = [[1.0, 1.0], [-1.0, -1.0], [1.0, 0.0], [2.0, 0.0], [np.nan, 0.0]]   # edges, outside, NaN
    real[:3] = [[1.0, -1.0], [0.125, 0.5], [-1.5, 0.0]]
    kl, counts = kl_score(torch.from_numpy(real).cuda(), torch.from_numpy(gen).cuda(), return_counts=True)
    cr, cg, ref = _ref(real, gen)
    assert np.array_equal(counts[0].cpu().numpy(), cr.astype(np.int32))
    assert np.array_equal(counts[1].cpu().numpy(), cg.astype(np.int32))
    assert abs(kl - ref) <= 1e-12 * max(1.0, abs(ref)), (kl, ref)


def test_kl_score_strided_subsample():
    from cglgan.evaluation import kl_score
    g = np.random.default_rng(1)
    real, gen = _ring(8000, g), _ring(3000, g, std=0.02)
    kl = kl_score(torch.from_numpy(real).cuda(), torch.from_numpy(gen).cuda(), num_sample=1000, num_servers=1)
    _, _, ref = _ref(real[::8000 // 1000], gen[::3000 // 1000])
    assert abs(kl - ref) <= 1e-12 * max(1.0, abs(ref))


def test_kl_score_two_servers_per_server_stride():
    """num_servers = 2 (CGLGAN/2DMG/main.py:75-80): each server's X is strided by
    len(X_s) // (num_sample // S) on its own, then the two samples are concatenated."""
    from cglgan.evaluation import kl_score
    g = np.random.default_rng(2)
    real = _ring(10000, g)
    x0, x1 = _ring(500, g, std=0.03), _ring(1500, g, std=0.06)
    kl = kl_score(torch.from_numpy(real).cuda(), [torch.from_numpy(x0).cuda(), torch.from_numpy(x1).cuda()],
                  num_sample=1000)
    d = np.concatenate([x0[::500 // 500], x1[::1500 // 500]], 0)
    _, _, ref = _ref(real[::10000 // 1000], d)
    assert abs(kl - ref) <= 1e-12 * max(1.0, abs(ref)), (kl, ref)
