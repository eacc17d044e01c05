"""Worker data shards of the reference drivers: the non-IID partitioner, the
data-size weights beta / A, and device-resident shards for the fused worker rounds.

``allocate_dataset`` restates the reference's module-level ``allocate_dataset(data, iid)`` as a pure
function of the labels and the driver's ``random.Random`` (``rd = Random(); rd.seed(20211212)``,
capgan.py:25-27), returning index arrays into the ORIGINAL dataset order instead of mutating a
torchvision dataset:

* variant ``"capgan"`` -- capgan.py:358-424 (= mixed-gan.py:400-468, CAPGAN/MNIST/*.py):
    test sample  ``rd.sample(range(n), num_sample)``                                    (:365)
    iid 0        ``rd.shuffle`` of all indices, N equal slices of int(n / N)            (:367-376)
    iid 1, 2     ``np.argsort(labels)`` (numpy's default sort, as the reference calls it), random
                 shard fractions from ``rd.sample(range(1, N^2), N - 1)`` cut points     (:378-387)
    iid 1        worker i draws int(size_i n) samples (capped) from the label window of classes
                 i-1, i, i+1 (wrapping), ``rd.sample`` of the window positions         (:389-411)
    iid 2        worker i draws from one class run (the next run after the previous worker's),
                 ``rd.sample(range(s, l), min(int(size_i n), l - s))``                  (:412-424)
* variant ``"ring"`` -- CGLGAN/2DMG/main.py:382-438 (the 2-D Gaussian-mixture driver): the same
  test sample / iid 0 / iid 1; iid 2 hands worker i the whole next class run, without sampling, and
  stops one element short of the end of the data (``l < len(data) - 1``, :433).

Parity: pinned against the reference's own ``allocate_dataset`` functions, executed on synthetic
label vectors by tests/golden/make_partition_golden.py (tests/golden/partition.json).  The order of
equal labels after ``np.argsort`` (quicksort, not stable) is whatever this host's numpy returns --
the same call the reference makes.
"""
from __future__ import annotations

from random import Random

import numpy as np
import torch

SEED = 20211212


def driver_rng(seed: int = SEED) -> Random:
    """The drivers' module-level generator: ``rd = Random(); rd.seed(seed)`` (capgan.py:25-27)."""
    rd = Random()
    rd.seed(seed)
    return rd


def _sizes(rd: Random, n_workers: int):
    se = rd.sample(range(1, n_workers ** 2), k=n_workers - 1)
    se.append(0)
    se.append(n_workers ** 2)
    se = sorted(se)
    return [(se[i] - se[i - 1]) / (n_workers ** 2) for i in range(1, len(se))]


def allocate_dataset(labels, iid: int, num_workers: int, num_class: int = 10, num_sample: int = 1000,
                     rd: Random | None = None, variant: str = "capgan"):
    """Returns ``(test_idx, shards, sizes)``: the test-sample indices, one int64 index array per worker
    (into the original order of ``labels``) and the shard fractions drawn (iid 0: 1/N each)."""
    if variant not in ("capgan", "ring"):
        raise ValueError("variant must be 'capgan' (capgan.py / mixed-gan.py) or 'ring' (CGLGAN/2DMG)")
    if iid not in (0, 1, 2):
        raise ValueError("iid must be 0 (iid), 1 (3-class windows) or 2 (one class per worker)")
    rd = rd if rd is not None else driver_rng()
    lab = np.asarray(labels.cpu().numpy() if torch.is_tensor(labels) else labels)
    n = len(lab)
    test_idx = np.asarray(rd.sample(range(n), num_sample), dtype=np.int64)
    shards = []
    if iid == 0:
        sizes = [1.0 / num_workers for _ in range(num_workers)]
        idx = list(range(n))
        rd.shuffle(idx)
        for frac in sizes:
            part = int(frac * n)
            shards.append(np.asarray(idx[:part], dtype=np.int64))
            idx = idx[part:]
        return test_idx, shards, sizes
    order = np.argsort(lab)
    slab = lab[order]
    sizes = _sizes(rd, num_workers)
    if iid == 1:
        ll = slab.tolist()
        for i in range(num_workers):
            s = ll.index((i - 1 + num_class) % num_class)
            e = ll.index((i + 2) % num_class)
            l = int(sizes[i] * n)
            if s < e:
                l = min(l, e - s)
                choose = rd.sample(range(s, e), l)
            else:
                l = min(l, e + n - s)
                choose = rd.sample(list(range(0, e)) + list(range(s, n)), l)
            shards.append(order[np.asarray(choose, dtype=np.int64)])
        return test_idx, shards, sizes
    if variant == "capgan":
        l, s = 1, 0
        for i in range(num_workers):
            while l < n and slab[l] == slab[l - 1]:
                l += 1
            choose = rd.sample(range(s, l), min(int(sizes[i] * n), l - s))
            shards.append(order[np.asarray(choose, dtype=np.int64)])
            s = l % n
            l = s + 1
        return test_idx, shards, sizes
    # ring iid 2: contiguous class runs, consumed from the front (CGLGAN/2DMG/main.py:431-438)
    rem_order, rem_lab = order, slab
    for i in range(num_workers):
        l = 1
        while rem_lab[l] == rem_lab[l - 1] and l < len(rem_order) - 1:
            l += 1
        shards.append(np.asarray(rem_order[:l], dtype=np.int64))
        rem_order, rem_lab = rem_order[l:], rem_lab[l:]
    return test_idx, shards, sizes


def beta_weights(shard_lens):
    """Server.run's data-size weights, float32 as the reference computes them (capgan.py:149-153):
    beta = zeros(N); beta[c] = len(dataset_c); data_len = beta.sum(); beta /= data_len."""
    b = torch.zeros(len(shard_lens))
    for c, v in enumerate(shard_lens):
        b[c] = float(v)
    data_len = b.sum()
    return (b / data_len), float(data_len)


def cloud_weights(server_data_lens):
    """The Cloud's FedAvg weights A_s = data_len_s / sum (float32, mixed-gan.py:105-110, capgan.py:100-105)."""
    a = torch.zeros(len(server_data_lens))
    for s, v in enumerate(server_data_lens):
        a[s] = float(v)
    return a / a.sum()


def eval_subsample(x: torch.Tensor, num_sample: int):
    """``test_set[::test_set.shape[0] // num_sample]`` / ``X[::X.shape[0] // (num_sample // S)]``
    (CGLGAN/2DMG/main.py:68, capgan.py:80): the evaluation subsample, a strided view."""
    return x[::max(1, x.shape[0] // num_sample)]


def gmm(num_class: int = 5, x: int = 10000, np_seed: int = SEED, generator: torch.Generator | None = None,
        device=None):
    """The 2-D Gaussian-mixture ring of CGLGAN/2DMG/data.py:5-38 (``gmm(n_class, x).data / .targets``):
    ``num_class`` modes at theta = linspace(0, 2 pi (1 - 1/n), n) on the unit circle (x = sin, y = cos),
    std 0.01, ``x * num_class`` points whose modes are drawn one by one with numpy's legacy generator
    (the reference seeds numpy's global generator with 20211212 at import, data.py:4 -- reproduced by
    ``np_seed``) and whose coordinates are one ``torch.normal`` call of 2 values per point from the
    torch CPU generator (the global one, as the reference, unless ``generator`` is given); then sorted by
    label with ``torch.sort``.  Returns ``(data [n, 2] float32, targets [n] float32)``.

    The draws are made on the host because their order IS the format (the same points as the
    reference for the same seeds: pinned by the sha256 in tests/golden/golden_steps.json ``ring_b64``);
    the result is moved to ``device`` once.  Generation is init-time work, not the round's hot path."""
    rs = np.random.RandomState(np_seed)
    thetas = np.linspace(0, 2 * (1 - 1 / num_class) * np.pi, num_class)
    xs, ys = np.sin(thetas), np.cos(thetas)
    n = x * num_class
    data = torch.zeros(n, 2)
    labels = torch.zeros(n)
    std = 0.01 * torch.ones(1, 2)
    means = [torch.Tensor([xs[c], ys[c]]) for c in range(num_class)]
    for i in range(n):
        coin = rs.randint(0, num_class)
        data[i, :] = torch.normal(mean=means[coin], std=std, generator=generator)
        labels[i] = coin
    targets, order = torch.sort(labels)
    data = data[order]
    if device is not None:
        data, targets = data.to(device), targets.to(device)
    return data, targets


def synthetic_mnist(n: int, num_class: int = 10, seed: int = 1, noise: float = 0.35, img_dim: int = 784,
                    device=None):
    """A labelled MNIST-shaped dataset for the driver and the benchmarks (there is no MNIST on these
    hosts): ``num_class`` fixed random prototype images, each sample = its class prototype
    + uniform noise, clamped to [-1, 1] (the range Normalize([0.5], [0.5]) gives, capgan.py:469).
    Labels are uniform, so ``allocate_dataset`` produces the reference's IID / non-IID shard shapes
    (SURVEY 8d C5).  Returns ``(images [n, img_dim] float32, labels [n] int64)``."""
    g = torch.Generator().manual_seed(seed)
    protos = torch.rand(num_class, img_dim, generator=g) * 2 - 1
    labels = torch.randint(0, num_class, (n,), generator=g)
    imgs = (protos[labels] + noise * (torch.rand(n, img_dim, generator=g) * 2 - 1)).clamp_(-1.0, 1.0)
    if device is not None:
        imgs, labels = imgs.to(device), labels.to(device)
    return imgs, labels


def sample_batches(shard: torch.Tensor, batch: int, count: int, seed: int):
    """``count`` real batches of ``batch`` rows drawn from a shard with DataLoader(shuffle=True,
    drop_last=False) semantics (capgan.py:282, 326-332): a fresh permutation per pass over the shard,
    the pass's last batch possibly short.  Host-side helper for explicit-input rounds (tests, driver
    replays); the fused round samples on the device."""
    g = torch.Generator().manual_seed(seed)
    n = shard.shape[0]
    out, perm, pos = [], torch.randperm(n, generator=g), 0
    while len(out) < count:
        if pos >= n:
            perm, pos = torch.randperm(n, generator=g), 0
        idx = perm[pos:pos + batch]
        pos += batch
        out.append(shard[idx.to(shard.device)])
    return out


def device_shard(images: torch.Tensor, idx, device="cuda") -> torch.Tensor:
    """One worker's shard resident in HBM as the fused rounds read it: [len, features] float32 rows
    of ``images`` (any [n, ...] tensor) in shard order, gathered once (the rounds then sample it
    every round on device, DataLoader(shuffle=True) semantics)."""
    ii = torch.as_tensor(np.asarray(idx), dtype=torch.long)
    rows = images.reshape(images.shape[0], -1)[ii].to(torch.float32)
    return rows.to(device).contiguous()
