"""Multi-round hipGraphs (cgl_gan_run_graph_rounds): K complete rounds captured back to back in
one graph launch must be exactly K single-round graph replays (and K eager rounds) -- every per-round value (z, the
real-batch sampler, Adam step counts, lambda, running statistics) comes from the device state the previous round
advanced.  Checked bitwise at the bench's B = 256 (z drawn on device, the in-graph sampler across a pass boundary),
and through WorkerExchange.rounds, the path bench.py times."""
import pytest
import torch

pytestmark = pytest.mark.gpu

KEYS = ("g_params", "g_m", "g_v", "g_running", "d_params", "d_m", "d_v", "d_grads", "g_grads")


def _step(B=256, rows=700):
    from cglgan import GanStep, specs
    from cglgan.init import default_init
    g = torch.Generator(device="cuda").manual_seed(1000)
    data = torch.rand(rows, 784, device="cuda", generator=g) * 2 - 1
    gm, dm = specs.mnist_generator(), specs.mnist_discriminator()
    st = GanStep(gm, dm, batch=B, batch_real=B, loss="ce", weighting="capgan", seed=20211212, gen_z=True, real=data,
                 sample_n=rows)
    torch.manual_seed(20211212)
    default_init(gm, st.g_views)
    torch.manual_seed(20211213)
    default_init(dm, st.d_views)
    st.reset()
    return st


def _same(a, b):
    torch.cuda.synchronize()
    for k in KEYS:
        x, y = getattr(a, k), getattr(b, k)
        assert torch.equal(x, y), (k, (x - y).abs().max().item())
    sa, sb = a.stats(), b.stats()
    for k in ("round", "d_loss", "g_loss", "lambda", "F", "bn_batches"):
        assert sa[k] == sb[k], (k, sa[k], sb[k])


def test_graph_rounds_equal_single_rounds():
    a, b, c = _step(), _step(), _step()
    # 2 + 5 + 3 + 7 + 5 + 11 rounds: four distinct counts in the cache, then an eviction (11), then a cached one
    counts = [2, 5, 3, 7, 5, 11]
    for n in counts:
        a.run_rounds(n)
    for _ in range(sum(counts)):
        b.run(graph=True)
        c.run(graph=False)
    _same(a, b)
    _same(a, c)
    # the sampler crossed pass boundaries (700 rows = 2 full batches + one of 188 per pass)
    assert a.stats()["round"] == sum(counts)


def test_exchange_rounds_path():
    from cglgan.exchange import WorkerExchange
    a, b = _step(), _step()
    ea, eb = WorkerExchange(a, None), WorkerExchange(b, None)
    a.prepare_rounds(4)
    ea.rounds(0, 4)
    ea.rounds(4, 4)
    ea.rounds(8, 1)
    for r in range(9):
        eb.round(r, graph=True)
    _same(a, b)


def test_state_written_between_graph_rounds():
    """A parameter write from outside the round (a state-dict load) between multi-round launches refreshes the
    packed copies exactly as before a single-round replay."""
    a, b = _step(), _step()
    a.run_rounds(3)
    for _ in range(3):
        b.run(graph=True)
    with torch.no_grad():
        for s in (a, b):
            s.g_views["model.0.weight"].mul_(0.5)
            s.d_views["model.0.weight"].mul_(0.5)
    a.run_rounds(4)
    for _ in range(4):
        b.run(graph=True)
    _same(a, b)
