"""Resume on the GPU steps (new): a step restored with load_resume_state from another step's
resume_state after round 2 -- including a step built with different initial weights and a fresh
device state -- runs rounds 3-4 bitwise as the uninterrupted step does (fixed-order reductions; the
round counter in the saved device state drives z, the sampler and the Adam bias corrections)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _mlp(seed_init):
    from cglgan import GanStep, specs
    from cglgan.init import default_init
    gm, dm = specs.mnist_generator(), specs.mnist_discriminator()
    g = torch.Generator().manual_seed(11)
    real = (torch.rand(300, 784, generator=g) * 2 - 1).cuda()
    st = GanStep(gm, dm, batch=64, epoch=2, gen_z=True, real=real, sample_n=300, seed=77)
    torch.manual_seed(seed_init)
    default_init(gm, st.g_views)
    default_init(dm, st.d_views)
    st.reset()
    return st


def test_gan_step_resume_bitwise():
    a, b = _mlp(1), _mlp(1)
    for t in range(2):
        a.run(graph=t == 1)
        b.run(graph=t == 1)
    sd = b.resume_state()
    c = _mlp(2)                       # other weights, round 0: everything must come from the file
    c.load_resume_state(sd)
    for t in range(2):
        a.run(graph=True)
        c.run(graph=t == 0)
    torch.cuda.synchronize()
    for k in ("g_params", "d_params", "g_m", "d_v", "g_running"):
        assert torch.equal(getattr(a, k), getattr(c, k)), k
    sa, sc = a.stats(), c.stats()
    assert sa["round"] == sc["round"] == 4 and sa["lambda"] == sc["lambda"] and sa["d_loss"] == sc["d_loss"]


def _conv(seed_init, graph):
    from cglgan.conv_step import ConvGanStep
    g = torch.Generator().manual_seed(5)
    data = (torch.rand(100, 1024, generator=g) * 2 - 1).cuda()
    st = ConvGanStep(32, data=data, seed=9, graph=graph)
    st.init_default(seed_init, seed_init + 1)
    return st


@pytest.mark.parametrize("graph", [False, True])
def test_conv_step_resume_bitwise(graph):
    a, b = _conv(1, graph), _conv(1, graph)
    for _ in range(2):
        a.run()
        b.run()
    sd = b.resume_state()
    c = _conv(3, graph)
    c.load_resume_state(sd)
    for _ in range(3):                # crosses the 100-row pass boundary of the sampler (32 per round)
        a.run()
        c.run()
    torch.cuda.synchronize()
    for k in ("p", "m", "v"):
        assert torch.equal(getattr(a.G, k), getattr(c.G, k)), ("G", k)
        assert torch.equal(getattr(a.D, k), getattr(c.D, k)), ("D", k)
    assert a.stats() == c.stats()
