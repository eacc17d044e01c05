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
        if phase == C.PHASE_B and self.exchange_mode == "gather":
            self._combine()
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

    def _alpha(self):
        l = self.losses_all.clone()
        if self.weighting == "capgan":
            a = O.capgan_alpha(self.lsgd.lam.detach(), l, self.beta)
            self.F = float((a * l).sum() - O.LAMBDA_REG * self.lsgd.lam.detach())
        else:
            a = torch.full((self.n_workers,), 1.0 / self.n_workers)
            self.F = float(l.mean())
        return a

    def alpha_scale(self):
        self._x.mul_(self._alpha()[self.rank])

    # the gathered exchange (GanStep.set_exchange("gather")): one all_gather of [gradient | loss | pad] slots,
    # then alpha and the rank-ordered weighted sum at the start of phase B (cgl_alpha_combine)
    exchange_mode = "reduce"

    def set_exchange(self, mode):
        self.exchange_mode = mode

    def gather_buffers(self):
        n = self._x.numel()
        self._slot = (n + 1 + 63) // 64 * 64
        send = torch.zeros(self._slot, dtype=self._x.dtype)
        send[:n] = self._x.flatten()
        send[n] = self.loss.detach()
        self._recv = torch.zeros(self.n_workers * self._slot, dtype=self._x.dtype)
        return send, self._recv

    def _combine(self):
        n = self._x.numel()
        g = self._recv.view(self.n_workers, self._slot)
        self.losses_all.copy_(g[:, n])
        a = self._alpha()
        tot = g[0, :n] * a[0]
        for q in range(1, self.n_workers):
            tot += g[q, :n] * a[q]
        self._x = tot.view_as(self._x).clone()

    def exchange_buffer(self):
        return self._x

    def g_params(self):
        return {k: v.detach().clone() for k, v in self.G.params.items()}


# ------------------------------------------------------------------------------------------------
def driver_inputs(cfg, server, rank, shard, r):
    """The explicit inputs of round ``r`` for the CPU driver stand-in (and the test's reference run):
    z shared by a server group, real batches per worker."""
    from cglgan.data import sample_batches
    g = torch.Generator().manual_seed(cfg.seed * 1000 + 97 * server + r)
    B = cfg.batch_size
    z1, z2 = torch.randn(B, 100, generator=g), torch.randn(B, 100, generator=g)
    reals = sample_batches(shard, B, cfg.epoch, seed=7 * 1000003 + 1009 * rank + r)
    return z1, z2, reals


class OracleDriverStep:
    """CPU stand-in for the GanStep a ``cglgan.driver.Driver`` builds (capgan / mixg / mdgan), on the
    oracle's arithmetic, with the state in flat buffers as the exchange sees them (``g_params``,
    ``trunk_slices()``, ``d_params``): lets the driver's topology (server groups, cloud group),
    WorkerExchange and its collectives run multi-process over gloo."""

    def __init__(self, cfg, topo, shard, beta, g_sd, d_sd):
        self.cfg, self.topo, self.shard = cfg, topo, shard
        self.n_workers, self.rank = topo.heads, topo.local
        self.weighting = cfg.weighting_
        self.mixg = cfg.algo == "mixg"
        if self.mixg:
            self.nets = [O.SeqNet(O.mnist_mixgen_trunk_spec()), O.SeqNet(O.mnist_mixgen_head_spec(topo.local))]
        else:
            self.nets = [O.SeqNet(O.mnist_generator_spec())]
        for n in self.nets:
            with torch.no_grad():
                for k, v in n.params.items():
                    v.copy_(g_sd[k])
        self.w = O.Worker(O.SeqNet(O.mnist_discriminator_spec(sigmoid=cfg.algo == "mdgan")),
                          "bce" if cfg.algo == "mdgan" else "ce")
        with torch.no_grad():
            for k, v in self.w.D.params.items():
                v.copy_(d_sd[k])
        self.gp = [p for n in self.nets for p in n.params.values()]
        self.gr = [b for n in self.nets for k, b in n.buffers.items() if "running" in k]
        self.trunk_np = sum(p.numel() for p in self.nets[0].params.values()) if self.mixg else None
        self.trunk_nr = sum(b.numel() for k, b in self.nets[0].buffers.items() if "running" in k) if self.mixg else 0
        self.opt_g = O.Adam(self.gp)
        self.lsgd = O.LambdaSGD()
        self.beta = torch.tensor(beta)
        self.losses_all = torch.zeros(self.n_workers)
        self.g_params = torch.cat([p.detach().flatten() for p in self.gp]).clone()
        self.g_running = torch.cat([b.flatten() for b in self.gr]).clone() if self.gr else torch.zeros(1)
        self.d_params = torch.cat([p.detach().flatten() for p in self.w.D.params.values()]).clone()
        self.round = 0
        self.F = None

    @staticmethod
    def _load(ts, flat):
        off = 0
        with torch.no_grad():
            for t in ts:
                t.copy_(flat[off:off + t.numel()].view_as(t))
                off += t.numel()

    def trunk_slices(self):
        return self.g_params[:self.trunk_np], (self.g_running[:self.trunk_nr] if self.trunk_nr else None)

    def run(self, phase=C.PHASE_ALL, graph=False):
        if phase in (C.PHASE_A, C.PHASE_ALL):
            self._load(self.gp, self.g_params)
            self._load(self.gr, self.g_running)
            self._load(list(self.w.D.params.values()), self.d_params)
            z1, z2, reals = driver_inputs(self.cfg, self.topo.server, self.topo.rank, self.shard, self.round)
            with torch.no_grad():
                xd = z1
                for n in self.nets:
                    xd = n.forward(xd)
            self._t2 = self.nets[0].forward(z2)
            hx = self._t2.detach().requires_grad_(True)
            xg = self.nets[1].forward(hx) if self.mixg else hx
            self.d_losses = [self.w.d_step(r, xd.clone(), half=(self.w.loss == "ce")) for r in reals]
            self.d_params = torch.cat([p.detach().flatten() for p in self.w.D.params.values()]).clone()
            self.loss = self.w.g_loss(xg)
            if self.mixg:     # phase 1 (mixed-gan.py:263-268): the head's gradient of its own loss
                hp = list(self.nets[1].params.values())
                gr = torch.autograd.grad(self.loss, [hx] + hp)
                self._x = gr[0].clone()
                self._head_grads = gr[1:]
            else:
                self._x = torch.autograd.grad(self.loss, hx)[0].clone()
        if phase == C.PHASE_ALL:
            self.losses_all.copy_(self.own_loss())
            self.alpha_scale()
        if phase in (C.PHASE_B, C.PHASE_ALL):
            for p in self.gp:
                p.grad = None
            self._t2.backward(self._x)
            if self.mixg:
                for p, g in zip(self.nets[1].params.values(), self._head_grads):
                    p.grad = g
            self.lsgd.zero_grad()
            if self.weighting != "mean":
                self.lsgd.lam.grad = torch.tensor(-O.LAMBDA_REG)   # dF/dlambda (capgan.py:249)
            self.lsgd.step()
            self.opt_g.step()
            self.g_params = torch.cat([p.detach().flatten() for p in self.gp]).clone()
            self.g_running = torch.cat([b.flatten() for b in self.gr]).clone() if self.gr else torch.zeros(1)
            self.round += 1

    def own_loss(self):
        return self.loss.detach().reshape(1).clone()

    def alpha_scale(self):
        import torch.nn.functional as F
        l, lam, b = self.losses_all.clone(), self.lsgd.lam.detach(), self.beta
        if self.weighting == "capgan":
            a = O.capgan_alpha(lam, l, b)
        elif self.weighting == "mix_single":
            a = F.softmax(b * lam * l, dim=0)
        elif self.weighting == "mix_double":
            a = F.softmax(b * F.softmax(lam * l, dim=0), dim=0)
        else:
            a = torch.full((self.n_workers,), 1.0 / self.n_workers)
        self.F = float((a * l).sum() - (0.0 if self.weighting == "mean" else O.LAMBDA_REG * float(lam)))
        self._x.mul_(a[self.rank])

    def exchange_buffer(self):
        return self._x

    def resume_state(self):
        """The stand-in's training state (GanStep.resume_state's role): flat G / running / D buffers,
        both Adams, lambda and the round counter that drives its inputs."""
        out = {"g_params": self.g_params.clone(), "g_running": self.g_running.clone(),
               "d_params": self.d_params.clone(), "round": torch.tensor(self.round),
               "lam": self.lsgd.lam.detach().clone()}
        for tag, opt in (("g", self.opt_g), ("d", self.w.opt)):
            for i, (m, v, st) in enumerate(zip(opt.m, opt.v, opt.step_t)):
                out[f"{tag}_m{i}"], out[f"{tag}_v{i}"], out[f"{tag}_t{i}"] = m.clone(), v.clone(), st.clone()
        return out

    @torch.no_grad()
    def load_resume_state(self, sd):
        self.g_params.copy_(sd["g_params"])
        self.g_running.copy_(sd["g_running"])
        self.d_params.copy_(sd["d_params"])
        self.round = int(sd["round"])
        self.lsgd.lam.copy_(sd["lam"])
        for tag, opt in (("g", self.opt_g), ("d", self.w.opt)):
            for i in range(len(opt.m)):
                opt.m[i].copy_(sd[f"{tag}_m{i}"])
                opt.v[i].copy_(sd[f"{tag}_v{i}"])
                opt.step_t[i].copy_(sd[f"{tag}_t{i}"])

    def stats(self):
        return {"round": self.round, "d_loss": [float(x) for x in self.d_losses], "g_loss": float(self.loss.detach()),
                "lambda": float(self.lsgd.lam), "F": self.F}


def oracle_step_factory(cfg, topo, shard, beta, g_sd, d_sd, device):
    return OracleDriverStep(cfg, topo, shard, beta, g_sd, d_sd)
