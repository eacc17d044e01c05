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


def device_shard(images: torch.Tensor, idx, device="cuda") -> torch.Tensor:
    """One worker's shard resident in HBM as the fused rounds read it: [len, features] float32 rows
    of ``images`` (any [n, ...] tensor) in shard order, gathered once (the rounds then sample it
    every round on device, DataLoader(shuffle=True) semantics)."""
    ii = torch.as_tensor(np.asarray(idx), dtype=torch.long)
    rows = images.reshape(images.shape[0], -1)[ii].to(torch.float32)
    return rows.to(device).contiguous()
