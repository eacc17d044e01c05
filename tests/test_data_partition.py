"""cglgan.data: the drivers' non-IID partitioner and data-size weights.

Pinned bit for bit against the reference's own ``allocate_dataset`` (capgan.py:358-424,
CGLGAN/2DMG/main.py:382-438) run on synthetic label vectors by tests/golden/make_partition_golden.py;
plus size-independent properties on an MNIST-sized label vector.
"""
import json
import os

import numpy as np
import pytest
import torch

from cglgan import data as D

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "partition.json")))


@pytest.mark.parametrize("case", GOLD["cases"], ids=lambda c: f"{c['variant']}-iid{c['iid']}-N{c['num_workers']}")
def test_partition_matches_reference(case):
    labels = np.asarray(GOLD[case["labels"]])
    test_idx, shards, _ = D.allocate_dataset(labels, case["iid"], case["num_workers"], case["num_class"],
                                             case["num_sample"], variant=case["variant"])
    assert test_idx.tolist() == case["test"]
    assert len(shards) == len(case["shards"])
    for got, exp in zip(shards, case["shards"]):
        assert got.tolist() == exp


def test_partition_properties_mnist_size():
    rs = np.random.RandomState(1)
    labels = rs.randint(0, 10, size=60000)
    _, sh0, s0 = D.allocate_dataset(labels, 0, 10)
    allidx = np.concatenate(sh0)
    assert len(allidx) == 60000 and len(np.unique(allidx)) == 60000 and s0 == [0.1] * 10
    _, sh1, s1 = D.allocate_dataset(labels, 1, 10)
    assert abs(sum(s1) - 1.0) < 1e-12
    for i, sh in enumerate(sh1):
        assert len(np.unique(sh)) == len(sh)
        assert set(np.unique(labels[sh])) <= {(i - 1) % 10, i, (i + 1) % 10}
    _, sh2, _ = D.allocate_dataset(labels, 2, 10)
    for i, sh in enumerate(sh2):
        assert len(np.unique(labels[sh])) <= 1
    beta, n = D.beta_weights([len(s) for s in sh1])
    assert beta.dtype == torch.float32 and abs(float(beta.sum()) - 1.0) < 1e-6
    assert n == float(sum(len(s) for s in sh1))


def test_weights_and_subsample():
    a = D.cloud_weights([300, 100])
    assert torch.equal(a, torch.tensor([0.75, 0.25]))
    x = torch.arange(1000)
    assert torch.equal(D.eval_subsample(x, 100), x[::10])
