"""Product-side data formats (CPU): the 2-D Gaussian-mixture ring generator (CGLGAN/2DMG/data.py:5-38)
pinned against the sha256 the reference's own ``gmm`` produced (tests/golden/golden_steps.json
``ring_b64``: ``torch.manual_seed(20211212); gmm(8, 2000)``), and the labelled synthetic MNIST-shaped
set the driver and benchmarks shard with ``allocate_dataset``."""
import torch

from cglgan.data import allocate_dataset, gmm, sample_batches, synthetic_mnist
from golden_replay import load_golden, sha


def test_gmm_ring_matches_reference_points():
    fx = load_golden()["ring_b64"]
    torch.manual_seed(20211212)
    data, targets = gmm(8, fx["config"]["n_points_per_class"])
    assert data.shape == (16000, 2) and data.dtype == torch.float32
    assert sha(data) == fx["data_sha256"]
    assert torch.equal(targets, torch.sort(targets).values)           # sorted by label (data.py:36)
    r = data.norm(dim=1)
    assert float((r - 1).abs().max()) < 0.06                          # 8 modes on the unit circle, std .01


def test_synthetic_mnist_shards():
    x, y = synthetic_mnist(4000, seed=3)
    assert x.shape == (4000, 784) and float(x.min()) >= -1 and float(x.max()) <= 1
    assert set(y.tolist()) == set(range(10))
    _, shards, sizes = allocate_dataset(y, iid=1, num_workers=8, num_sample=100)
    assert len(shards) == 8
    for i, s in enumerate(shards):   # iid 1: worker i sees the class window i-1, i, i+1 (capgan.py:389-411)
        assert set(y[torch.as_tensor(s)].tolist()) <= {(i - 1) % 10, i % 10, (i + 1) % 10}
    b = sample_batches(x[torch.as_tensor(shards[0])], 64, 5, seed=1)
    assert all(t.shape[1] == 784 for t in b) and b[0].shape[0] == 64
