"""WorkerExchange's choice of exchange form:
* exchange="auto" falls back to the reduce form when the step has no gathered form (the combine head is planned
  only when the exchange tensor holds a multiple of 4 floats: a 2-D ring generator at an odd batch), instead of
  failing in the constructor; an explicit "gather" there still raises;
* the library's mode is set for both forms, so a reduce-form exchange built on a step that a gathered-form
  exchange used before runs the reduce form (no combine over a stale gather buffer).
Each configuration runs split rounds through a one-rank loopback group and must equal the unsplit rounds bitwise."""
import pytest
import torch

pytestmark = pytest.mark.gpu


class Loopback:
    """A one-rank group: all_gather copies, the sums are the identity."""
    rank, size, capturable = 0, 1, False

    def all_gather(self, out, inp):
        out.copy_(inp)

    def all_reduce_sum(self, t):
        pass

    def all_reduce_mean(self, t, weights=None):
        pass


def _ring(B, seed=3):
    from cglgan import GanStep, specs
    from cglgan.data import gmm
    from cglgan.init import default_init
    torch.manual_seed(seed)
    data, _ = gmm(8, 200, device="cuda")
    gm, dm = specs.ring_generator(0), specs.ring_discriminator()
    st = GanStep(gm, dm, batch=B, loss="bce", weighting="cglgan", n_workers=1, rank=0, gen_z=True, real=data,
                 sample_n=data.shape[0], seed=91)
    torch.manual_seed(20211212)
    default_init(gm, st.g_views)
    default_init(dm, st.d_views)
    st.reset()
    return st


def _same(a, b):
    torch.cuda.synchronize()
    for k in ("g_params", "g_m", "g_v", "d_params", "d_m", "d_v"):
        x, y = getattr(a, k), getattr(b, k)
        assert torch.equal(x, y), (k, (x - y).abs().max().item())
    assert a.stats()["g_loss"] == b.stats()["g_loss"]


@pytest.mark.parametrize("B,want", [(63, "reduce"), (64, "gather")])
def test_auto_falls_back_to_reduce(B, want):
    from cglgan.exchange import WorkerExchange
    a, b = _ring(B), _ring(B)
    ex = WorkerExchange(a, Loopback(), force_split=True)
    assert ex.exchange == want and a.exchange_mode == want
    ref = WorkerExchange(b, None)
    for r in range(3):
        ex.round(r, graph=(r > 0))
        ref.round(r, graph=(r > 0))
    _same(a, b)


def test_explicit_gather_without_combine_raises():
    from cglgan.exchange import WorkerExchange
    with pytest.raises(RuntimeError):
        WorkerExchange(_ring(63), Loopback(), exchange="gather")


def test_mode_reset_between_exchanges():
    from cglgan.exchange import WorkerExchange
    a, b = _ring(64), _ring(64)
    g = WorkerExchange(a, Loopback(), force_split=True, exchange="gather")
    ref = WorkerExchange(b, None)
    for r in range(2):
        g.round(r, graph=True)
        ref.round(r, graph=True)
    red = WorkerExchange(a, Loopback(), force_split=True, exchange="reduce")
    assert a.exchange_mode == "reduce"
    for r in range(2, 5):
        red.round(r, graph=True)
        ref.round(r, graph=True)
    _same(a, b)
