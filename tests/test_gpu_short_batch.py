"""The in-graph sampler's short final batch (capgan.py:282, 326-331).

The reference's worker iterates ``DataLoader(dataset, batch_size, shuffle=True)``: every pass over its
shard ends with a batch of ``len(shard) mod batch_size`` rows, whose CE targets are sized by
``imgs.shape[0]``, and the next ``next()`` raises StopIteration and starts a freshly shuffled pass.
cglgan.GanStep(sample_n = len(shard)) runs that on the device: the round prologue writes the real-row
indices of each local D step and its real row count (cgl_gan_tensor 3 / 4), and the loss head takes
the real segment's size from the device (rows past it carry no loss and no gradient).

Checked here on a non-multiple shard cut by allocate_dataset(iid=1) (capgan.py:358-424):
  * the indices / row counts equal a host restatement of the sampler (keyed Feistel permutation per
    pass, batches cut in order, the last one short), and each pass visits every shard row once;
  * every round -- the ones before, at and after the pass boundary -- equals the CPU oracle's
    CapganServer.round on the same z and the same real batches (the short one as a short tensor):
    losses within the trajectory tolerance of test_gpu_step, the D parameters after the short-batch
    D step within 1e-4 relative (fp32 reduction order over three rounds).
Parity of the permutation itself is unpinned (the reference draws torch.randperm on the host; any
uniform shuffle is the reference's behaviour in distribution)."""
import numpy as np
import pytest
import torch

from parity_helpers import TRAJ_TOL, make_pair_oracle_only, rel_scalar

pytestmark = pytest.mark.gpu
M32 = 0xFFFFFFFF
B, EPOCH, SEED = 64, 2, 20211212


def _hash(x, k):
    x ^= k
    x = (x * 0x7FEB352D) & M32
    x ^= x >> 15
    x = (x * 0x846CA68B) & M32
    x ^= x >> 16
    return x


def _permute(i, n, key):
    """cgl_permute (csrc/cgl_common.h): 4-round Feistel on the smallest even bit width >= log2 n,
    cycle-walked into [0, n)."""
    bits = 2
    while (1 << bits) < n:
        bits += 1
    bits += bits & 1
    hb = bits // 2
    mask = (1 << hb) - 1
    x = i
    while True:
        l, r = x >> hb, x & mask
        for rnd in range(4):
            t = l ^ (_hash(r, (key + 0x9E3779B9 * (rnd + 1)) & M32) & mask)
            l, r = r, t
        x = (l << hb) | r
        if x < n:
            return x


def host_sampler(n, br, epoch, rnd, seed):
    """(indices [epoch][br], real rows [epoch]) of round ``rnd`` (0-based) -- cgl_round_prologue."""
    sseed = (seed ^ 0x5BD1E995) & M32
    nb = (n + br - 1) // br
    idx, rows = np.zeros((epoch, br), np.int64), np.zeros(epoch, np.int64)
    for e in range(epoch):
        bpos = rnd * epoch + e
        p, b = bpos // nb, bpos % nb
        key = sseed ^ ((p * 0x85EBCA6B + 0x1234567) & M32)
        rows[e] = min(br, n - b * br)
        for r in range(br):
            j = b * br + r
            idx[e, r] = _permute(j if j < n else n - 1, n, key)
    return idx, rows


def _shard():
    from cglgan.data import allocate_dataset, driver_rng, synthetic_mnist
    x, y = synthetic_mnist(3000, 10, seed=3)
    _, shards, _ = allocate_dataset(y, 1, 8, 10, 100, rd=driver_rng(11))
    for s in shards:
        if 3 * B < len(s) < 6 * B and len(s) % B:
            return x[torch.as_tensor(s)].reshape(len(s), -1)
    raise AssertionError(f"no shard of (3B, 6B) rows with a short batch: {[len(s) for s in shards]}")


def test_sampler_short_batch_pass_boundary():
    from cglgan import GanStep, specs
    real = _shard().float()
    n = real.shape[0]
    nb = (n + B - 1) // B
    srv, workers = make_pair_oracle_only("capgan")
    step = GanStep(specs.mnist_generator(), specs.mnist_discriminator(), batch=B, epoch=EPOCH, loss="ce",
                   weighting="capgan", seed=SEED, gen_z=True, real=real.cuda(), sample_n=n)
    step.load_state_dicts(srv.G.state_dict(), workers[0].D.state_dict())
    step.reset()
    rounds = (nb + EPOCH - 1) // EPOCH + 1          # past the first pass boundary
    seen = [[] for _ in range(rounds * EPOCH // nb + 1)]
    short_seen = False
    for t in range(rounds):
        step.run(graph=(t % 2 == 1))
        torch.cuda.synchronize()
        idx = step.internal(3).view(torch.int32).view(EPOCH, B).cpu().numpy()
        rows = step.internal(4).view(torch.int32)[:EPOCH].cpu().numpy()
        hidx, hrows = host_sampler(n, B, EPOCH, t, SEED)
        assert np.array_equal(rows, hrows), (t, rows, hrows)
        for e in range(EPOCH):
            assert np.array_equal(idx[e, :rows[e]], hidx[e, :rows[e]]), (t, e)
            seen[(t * EPOCH + e) // nb].extend(idx[e, :rows[e]].tolist())
            short_seen |= bool(rows[e] < B)
        z = step.z.cpu()
        reals = [real[torch.as_tensor(idx[e, :rows[e]], dtype=torch.long)] for e in range(EPOCH)]
        st = step.stats()
        r = srv.round(workers, z[:B], z[B:], [reals], weighting="capgan")
        for e in range(EPOCH):
            assert rel_scalar(st["d_loss"][e], r["d_losses"][e]) <= TRAJ_TOL, (t, e, st["d_loss"], r["d_losses"])
        assert rel_scalar(st["g_loss"], r["g_losses"][0]) <= TRAJ_TOL, (t, st["g_loss"], r["g_losses"])
        if any(rows < B):
            for k, v in step.d_views.items():
                o = workers[0].D.params[k].detach()
                err = float((v.cpu() - o).norm()) / max(float(o.norm()), 1e-30)
                assert err <= 1e-4, (t, k, err)
    assert short_seen
    # the first pass visited every row exactly once
    assert sorted(seen[0]) == list(range(n))
