"""Shared helpers for the GPU parity tests: build an oracle run and the HIP GanStep from the
same seeded initial state and inputs, and compare them with the tolerances SURVEY F8 sets
(single step <= 1e-5 relative; <= 10-step trajectory <= 1e-4 relative).
"""
import torch

from cglgan import GanStep, specs
from oracle import gan_oracle as O

STEP_TOL = 1e-5     # single step from identical state: losses, grads, updated params
TRAJ_TOL = 1e-4     # free-running trajectory, <= 10 steps


def rel(a, b):
    a = a.detach().double().cpu().flatten()
    b = b.detach().double().cpu().flatten()
    return float((a - b).norm() / max(b.norm(), 1e-30))


def rel_scalar(a, b):
    return abs(float(a) - float(b)) / max(abs(float(b)), 1e-30)


def make_pair(kind, B, Br=None, epoch=1, n_heads=2, head=0, seed=20211212, gen_z=False):
    """(oracle server, oracle workers, HIP step) with identical initial parameters."""
    if kind == "capgan":
        G, workers = O.build_capgan(1)
        srv = O.CapganServer(G, torch.tensor([1.0]))
        gm, dm, loss, weighting, xl = specs.mnist_generator(), specs.mnist_discriminator(), "ce", "capgan", -1
        gsd = G.state_dict()
    elif kind == "mdgan":
        G, workers = O.build_capgan(1, loss="bce")
        srv = O.CapganServer(G, torch.tensor([1.0]))
        gm, dm, loss, weighting, xl = specs.mnist_generator(), specs.mnist_discriminator(True), "bce", "mean", -1
        gsd = G.state_dict()
    elif kind == "ring":
        G, workers = O.build_ring(1, 1)
        srv = O.CglganServer(G, torch.tensor([1.0]))
        gm, dm, loss, weighting, xl = specs.ring_generator(0), specs.ring_discriminator(), "bce", "cglgan", -1
        gsd = G.state_dict()
    elif kind == "mixg1":
        # Mix-G with a single head: the full reference two-phase backward on one worker
        G, workers = O.build_mixg(1)
        srv = O.MixgServer(G, torch.tensor([1.0]))
        gm, dm, loss, weighting, xl = (specs.mixgen_worker(0), specs.mnist_discriminator(), "ce", "mix_single",
                                       specs.MIXGEN_HEAD_LAYER)
        gsd = G.state_dict()
    else:
        raise ValueError(kind)
    step = GanStep(gm, dm, batch=B, batch_real=Br or B, epoch=epoch, loss=loss, weighting=weighting,
                   exchange_layer=xl, seed=seed, gen_z=gen_z)
    step.load_state_dicts(gsd, workers[0].D.state_dict())
    step.reset()
    return srv, workers, step


def feed(step, z1, z2, reals):
    """Copy one round's explicit inputs into the step's device buffers."""
    step.z[: step.B].copy_(z1)
    step.z[step.B:].copy_(z2)
    step.real.copy_(torch.cat([r.reshape(r.shape[0], -1) for r in reals], 0))


def oracle_round(kind, srv, workers, z1, z2, reals):
    if kind in ("capgan",):
        return srv.round(workers, z1, z2, [reals], weighting="capgan")
    if kind == "mdgan":
        return srv.round(workers, z1, z2, [reals], weighting="mean")
    return srv.round(workers, z1, z2, [reals])


def inputs(kind, B, Br, epoch, seed):
    if kind == "ring":
        g = torch.Generator().manual_seed(seed)
        z1 = torch.randn(B, 100, generator=g)
        z2 = torch.randn(B, 100, generator=g)
        reals = [torch.randn(Br, 2, generator=g) * 0.7 for _ in range(epoch)]
        return z1, z2, reals
    z1, z2, reals = O.synthetic_inputs(B, 1, epoch, seed=seed, B_real=Br)
    return z1, z2, reals[0]
