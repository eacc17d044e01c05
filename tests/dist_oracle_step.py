"""CPU stand-in for ``cglgan.GanStep`` built on the oracle (TEST INFRASTRUCTURE ONLY).

It exposes exactly the surface ``cglgan.exchange.WorkerExchange`` drives -- ``run(phase)``,
``own_loss()``, ``losses_all``, ``alpha_scale()``, ``exchange_buffer()``, ``d_params``,
``n_workers`` -- so the multi-process exchange logic (collectives, alpha weighting, E-share)
can be exercised with the ``gloo`` backend on CPU and compared with the single-process oracle
in which the reference's Server backpropagates F_max through every worker's D (capgan.py:258).
"""
import torch

from cglgan import _lib as C
from oracle import gan_oracle as O


class OracleWorkerStep:
    def __init__(self, n_workers, rank, loss="ce", weighting="capgan", beta=None, seed=O.SEED):
        G, workers = O.build_capgan(n_workers, seed=seed, loss=loss)
        self.G, self.w = G, workers[rank]
        self.n_workers, self.rank = n_workers, rank
        self.weighting = weighting
        self.opt_g = O.Adam(G.parameters())
        self.lsgd = O.LambdaSGD()
        self.beta = torch.full((n_workers,), 1.0 / n_workers) if beta is None else torch.tensor(beta)
        self.losses_all = torch.zeros(n_workers)
        self.d_keys = list(self.w.D.params.keys())
        self.d_params = torch.cat([self.w.D.params[k].detach().flatten() for k in self.d_keys]).clone()
        self.F = None

    def set_inputs(self, z1, z2, real):
        self.z1, self.z2, self.real = z1, z2, real

    def _load_d(self):
        off = 0
        with torch.no_grad():
            for k in self.d_keys:
                p = self.w.D.params[k]
                p.copy_(self.d_params[off:off + p.numel()].view_as(p))
                off += p.numel()

    def _store_d(self):
        self.d_params = torch.cat([self.w.D.params[k].detach().flatten() for k in self.d_keys]).clone()

    def run(self, phase=C.PHASE_ALL, graph=False):
        if phase in (C.PHASE_A, C.PHASE_ALL):
            self._load_d()
            with torch.no_grad():
                xd = self.G.forward(self.z1)
            self.Xg = self.G.forward(self.z2)
            self.w.d_step(self.real, xd, half=(self.w.loss == "ce"))
            self._store_d()
            xg = self.Xg.detach().clone().requires_grad_(True)
            self.loss = self.w.g_loss(xg)
            self.loss.backward()
            self._x = xg.grad.detach().clone()
        if phase == C.PHASE_ALL:
            self.losses_all.copy_(self.own_loss())
            self.alpha_scale()
        if phase in (C.PHASE_B, C.PHASE_ALL):
            self.G.zero_grad()
            self.Xg.backward(self._x)
            self.lsgd.zero_grad()
            if self.weighting == "capgan":
                self.lsgd.lam.grad = torch.tensor(-O.LAMBDA_REG)   # dF/dlambda (capgan.py:249)
            self.lsgd.step()
            self.opt_g.step()

    def own_loss(self):
        return self.loss.detach().reshape(1).clone()

    def alpha_scale(self):
        l = self.losses_all.clone()
        if self.weighting == "capgan":
            a = O.capgan_alpha(self.lsgd.lam.detach(), l, self.beta)
            self.F = float((a * l).sum() - O.LAMBDA_REG * self.lsgd.lam.detach())
        else:
            a = torch.full((self.n_workers,), 1.0 / self.n_workers)
            self.F = float(l.mean())
        self._x.mul_(a[self.rank])

    def exchange_buffer(self):
        return self._x

    def g_params(self):
        return {k: v.detach().clone() for k, v in self.G.params.items()}
