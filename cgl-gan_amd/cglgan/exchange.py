"""Cross-worker exchange of one communication round, one worker per GPU.

The reference runs every role as a thread on one device and passes tensors (with their
autograd graph) through queue.Queue.  Here each worker is a process on its own
GPU, G is replicated (identical init, identical z stream, deterministic kernels), and the
round's queue traffic becomes collectives:

  CAPGAN / MDGAN / CGLGAN (capgan.py:223-259):
    phase A      local D step(s), G loss through the updated D, its gradient w.r.t. Xg
    all_gather   the N scalar G losses                      (Worker -> Server, capgan.py:347,228-232)
    alpha        lambda-weighting on device, own gradient scaled by alpha_rank (capgan.py:247-248)
    all_reduce   sum of alpha_i dl_i/dXg  [B, 784]           (F_max.backward through every D, :258)
    phase B      replicated G backward + Adam, lambda SGD    (:258-260)
  Mix-G (mixed-gan.py:238-292): the same with the trunk-output gradient [B, 512] inside a
    server group, plus the Cloud's data-size-weighted trunk average every cloud_epoch rounds
    (mixed-gan.py:104-124, 193-200; the reference's load of it is a no-op, SURVEY F4, kept
    reproducible with ``fedavg_compat_noop``).
  Gathered form (``exchange="gather"``, the default for groups of up to GATHER_MAX_WORKERS): ONE
    all_gather of every worker's [gradient | loss] slot replaces the loss all_gather, alpha and the
    gradient all_reduce; phase B starts with the alpha + rank-ordered weighted sum on device
    (cgl_gan_exchange_mode), so the sum no longer depends on the collective's reduction order.
  E-share (new behaviour): mean of the D parameters every E rounds.
  D-swap (MD-GAN, MDGAN/MNIST/mdgan.py:158-164, 258-262 -- commented out in the reference, parity
    unpinned): every E rounds the server shuffles the N discriminators with Random(server + 100) and
    worker i continues with D_{perm[i]}; here one point-to-point send/recv pair per rank over RCCL.

``DistComm`` wraps torch.distributed (backend "nccl" = RCCL over xGMI on MI355X, "gloo" on
CPU); ``LocalComm`` runs N workers of one process in lockstep (single-GPU rehearsal and
tests).  Both expose the same three collectives, so ``WorkerExchange`` is written once.
"""
from __future__ import annotations

import os
import random

import torch
import torch.distributed as dist

from . import _lib as C


# Largest group that takes the gathered exchange by default: each rank receives (N - 1) gradient slots (N = 8:
# 5.6 MB of a B = 256 round) where the ring all-reduce moves 2 (N - 1) / N of one (1.4 MB); up to 4 workers the
# removed loss all_gather and alpha launch outweigh the extra bytes on xGMI, beyond that the reduce form is kept.
GATHER_MAX_WORKERS = 4


class DistComm:
    """Collectives of one process group (this process = one worker)."""

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.size = dist.get_world_size(group)
        # RCCL collectives can be captured into a graph (WorkerExchange.round_graph); gloo's cannot
        self.capturable = dist.get_backend(group) == "nccl"

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor):
        dist.all_gather_into_tensor(out, inp, group=self.group)

    def all_reduce_sum(self, t: torch.Tensor):
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)

    def all_reduce_min(self, t: torch.Tensor):
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)

    def all_reduce_mean(self, t: torch.Tensor, weights=None):
        """sum_i w_i t_i (w = 1/N when None); identical result on every rank.  The plain mean is the sum divided by
        N on every backend (RCCL's ReduceOp.AVG computes sum(x_i * (1/N)), which is not the gloo / LocalComm value
        for N not a power of two); the division is one captured launch inside the whole-round graph."""
        if weights is not None:
            t.mul_(float(weights[self.rank]))
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
            t.div_(self.size)

    def swap(self, tensors, perm):
        """tensors <- the same tensors of rank perm[rank] (one isend / irecv pair per tensor)."""
        src, dst = perm[self.rank], perm.index(self.rank)
        if src == self.rank:
            return
        bufs = [torch.empty_like(t) for t in tensors]
        g = lambda r: dist.get_global_rank(self.group, r) if self.group is not None else r
        ops = []
        for t, b in zip(tensors, bufs):
            ops.append(dist.P2POp(dist.isend, t.contiguous(), g(dst), self.group))
            ops.append(dist.P2POp(dist.irecv, b, g(src), self.group))
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        for t, b in zip(tensors, bufs):
            t.copy_(b)


class DSwap:
    """The MD-GAN server's D shuffle (MDGAN/MNIST/mdgan.py:122-123,158-164): Random() seeded with
    server_rank + 100, ``shuffle`` of the N workers' discriminators; worker i receives D_{perm[i]}.
    Every rank holds the same seeded generator, so all ranks agree on perm without communication."""

    def __init__(self, n, server_rank=0):
        self.n = n
        self.rd = random.Random()
        self.rd.seed(server_rank + 100)

    def next_perm(self):
        p = list(range(self.n))
        self.rd.shuffle(p)
        return p


class WorkerExchange:
    """One worker's communication round (phase A -> collectives -> phase B).

    ``share_every`` > 0: E-share of the D parameters every that many rounds (a19).
    ``swap_every`` > 0: the MD-GAN D-swap inside the group every that many rounds, drawn by server
    ``server_rank``'s generator.
    ``cloud``/``cloud_every``: Cloud FedAvg across server groups (a18) with data-size weights
    ``cloud_weights`` (one per member of the cloud group), after every ``cloud_every``-th round;
    or, with ``cloud_due(r)`` (see ``mixg_cloud_due`` / ``capgan_cloud_due``), before round r as the
    reference's Server.run does.  ``cloud_scope``: "trunk" -- the Mix-G trunk parameters + running
    statistics (mixed-gan.py:193-200); "all" -- every G parameter, no buffers (CAPGAN's fedlab
    serialize_model / fedavg_aggregate / deserialize_model, capgan.py:169-175).  ``segema``: the
    result is segema * own + (1 - segema) * average (capgan.py:174, mixed-gan.py:198-199).
    """

    def __init__(self, step, comm=None, share_every: int = 0, cloud=None, cloud_every: int = 0,
                 cloud_weights=None, fedavg_compat_noop: bool = False, swap_every: int = 0,
                 cloud_scope: str = "trunk", segema: float = 0.0, cloud_due=None, server_rank: int = 0,
                 force_split: bool = False, exchange: str = "auto"):
        self.step = step
        self.comm = comm
        # test hook: take the N > 1 path (phase A, collectives, phase B) even in a one-rank group, so a
        # one-GPU box can run the exchange over real RCCL (two ranks cannot share a GPU under RCCL)
        self.force_split = force_split
        self.share_every = share_every
        self.swap_every = swap_every
        # the server's own generator: Random() seeded with server_rank + 100 (MDGAN/MNIST/mdgan.py:122-123)
        self.dswap = DSwap(comm.size, server_rank) if (comm is not None and swap_every > 0) else None
        self.cloud, self.cloud_every = cloud, cloud_every
        self.cloud_weights = cloud_weights
        self.fedavg_compat_noop = fedavg_compat_noop
        if cloud_scope not in ("trunk", "all"):
            raise ValueError("cloud_scope must be 'trunk' (Mix-G) or 'all' (CAPGAN)")
        self.cloud_scope, self.segema, self.cloud_due = cloud_scope, float(segema), cloud_due
        n = comm.size if comm is not None else 1
        if n != step.n_workers:
            raise ValueError(f"step planned for {step.n_workers} workers, group has {n}")
        if exchange not in ("auto", "gather", "reduce"):
            raise ValueError("exchange must be 'auto', 'gather' or 'reduce'")
        auto = exchange == "auto"
        if auto:
            exchange = "gather" if n <= GATHER_MAX_WORKERS and hasattr(step, "set_exchange") else "reduce"
        if comm is not None and hasattr(step, "set_exchange"):
            # the library's mode is set for BOTH forms: a step keeps its mode, so a later exchange in the other form
            # must not run phase B's combine over a stale gather buffer
            try:
                step.set_exchange(exchange)
            except RuntimeError:
                # the gathered form needs the combine head, planned only when the exchange tensor's size is a
                # multiple of 4 floats (cgl_gan_exchange_mode returns CGL_E_STATE otherwise): auto falls back
                if not (auto and exchange == "gather"):
                    raise
                exchange = "reduce"
                step.set_exchange(exchange)
        self.exchange = exchange
        # whole-round graph (graph=True rounds without a D-swap): phase A, this rank's collective(s) and phase B
        # captured as ONE torch CUDA graph once a split round has run eagerly through the group (RCCL's
        # communicator and buffers exist), replayed after -- the library's two graph launches, the collective
        # calls and (reduce form) the alpha launch leave the host path.  Only over a capturable group (RCCL);
        # CGL_ROUND_GRAPH=0 keeps the split path.  The first replay of each captured form is checked against the
        # split path on the same state (``_verify_round_graph``: bitwise, agreed over the group), so a stack whose
        # captured collectives misbehave falls back to the split rounds instead of training on wrong values.
        self.round_graph = (os.environ.get("CGL_ROUND_GRAPH", "1") != "0" and
                            bool(getattr(comm, "capturable", False)) and hasattr(step, "g_params") and
                            step.g_params.is_cuda)
        self._rgraph, self._split_ran = {}, False
        self.round_graph_checks = []      # (share, local verdict, group verdict) of every verification run
        self._rgraph_verified = set()
        # D's exchange (E-share / D-swap) after phase B on the main stream (default), or on a side stream beside
        # phase B (CGL_DX_SIDE=1).  Measured at world 1: the side branch slows every phase-B launch it runs beside
        # (+64 us per round for a ~15 us exchange, tests/rccl_world1_worker.py --time); serial it costs its own time.
        self.d_side = os.environ.get("CGL_DX_SIDE", "0") != "0"

    def exchange_mid(self):
        """The collectives between phase A and phase B of one round (this rank's side)."""
        s = self.step
        if self.exchange == "gather":
            send, recv = s.gather_buffers()
            self.comm.all_gather(recv, send)
        else:
            self.comm.all_gather(s.losses_all, s.own_loss())
            s.alpha_scale()
            self.comm.all_reduce_sum(s.exchange_buffer())

    def round(self, r: int, graph: bool = True):
        s = self.step
        if self.cloud is not None and self.cloud_due is not None and self.cloud_due(r):
            self.cloud_average()
        share = self.comm is not None and self.share_every > 0 and (r + 1) % self.share_every == 0
        swap = self.dswap is not None and (r + 1) % self.swap_every == 0
        if self.comm is None or (self.comm.size == 1 and not self.force_split):
            s.run(C.PHASE_ALL, graph=graph)
        elif graph and self.round_graph and self._split_ran and not swap and self._ensure_round_graph(share):
            if share in self._rgraph_verified:
                s._packed_current()          # (host-side check of the packed weight copies, as s.run does)
                self._rgraph[share].replay()
            else:
                self._verify_round_graph(r, share)
            share = False                # (the E-share ran inside the graph, or inside the verified split round)
        else:
            self._split_round(r, share, swap, graph)
            share = swap = False
        self._d_exchange(r, share, swap)
        if (self.cloud is not None and self.cloud_due is None and self.cloud_every > 0 and
                (r + 1) % self.cloud_every == 0):
            self.cloud_average()

    def rounds(self, r0: int, n: int, graph: bool = True):
        """Rounds r0 .. r0 + n - 1.  A worker with no group and no Cloud step (N = 1) runs them as multi-round graphs
        (GanStep.run_rounds); otherwise round by round."""
        if n <= 0:
            return
        if self.comm is None and self.cloud is None and graph and hasattr(self.step, "run_rounds"):
            self.step.run_rounds(n, graph=True)
            return
        for r in range(r0, r0 + n):
            self.round(r, graph=graph)

    def _split_round(self, r, share, swap, graph):
        """Phase A, the collective(s), phase B as separate calls, then D's exchange (E-share / D-swap)."""
        s = self.step
        self._split_ran = True
        s.run(C.PHASE_A, graph=graph)
        self.exchange_mid()
        side = self._side_stream() if ((share or swap) and self.d_side) else None
        if side is not None:
            # phase B (G backward + Adam G) never touches D: the E-share all-reduce / D-swap of
            # this round's updated D run on a side stream concurrently with it (issued in the
            # same order on every rank), joined before the next round's D step
            main = torch.cuda.current_stream()
            side.wait_stream(main)
            with torch.cuda.stream(side):
                self._d_exchange(r, share, swap)
            s.run(C.PHASE_B, graph=graph)
            main.wait_stream(side)
        else:
            s.run(C.PHASE_B, graph=graph)
            self._d_exchange(r, share, swap)

    _STATE = ("g_params", "g_grads", "g_m", "g_v", "g_running", "d_params", "d_grads", "d_m", "d_v", "losses_all",
              "workspace")
    _COMPARED = ("g_params", "g_m", "g_v", "g_running", "d_params", "d_m", "d_v")

    @torch.no_grad()
    def _verify_round_graph(self, r, share):
        """First use of a captured whole-round graph: round r runs through the split path (the reference form), the
        step's buffers are put back, the graph replays round r, and the two end states are compared bitwise (G, D,
        both Adams' moments, the running statistics, the round's losses).  Every rank of the group must agree
        (MIN-all-reduce of the verdict) before the graph is used; otherwise the split result is restored and the
        whole-round graph is turned off for this exchange.  Costs one extra round's work, once per captured form."""
        s = self.step
        s._packed_current()
        before = {k: getattr(s, k).clone() for k in self._STATE}
        self._split_round(r, share, False, True)
        split = {k: getattr(s, k).clone() for k in self._STATE}
        st_split = s.stats()
        for k in self._STATE:
            getattr(s, k).copy_(before[k])
        s.sync_params()                   # (the restored parameters' packed copies and the next z)
        self._rgraph[share].replay()
        st_graph = s.stats()
        ok = all(torch.equal(getattr(s, k), split[k]) for k in self._COMPARED)
        ok = ok and all(st_graph[k] == st_split[k] for k in ("round", "d_loss", "g_loss", "lambda", "F"))
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=s.g_params.device)
        self.comm.all_reduce_min(flag)
        ok_all = bool(flag.item())
        self.round_graph_checks.append((share, ok, ok_all))
        if ok_all:
            self._rgraph_verified.add(share)
            return
        import warnings
        warnings.warn("whole-round graph replay differs from the split round on this stack (local %s): split rounds "
                      "from now on" % ok)
        for k in self._STATE:
            getattr(s, k).copy_(split[k])
        s.sync_params()
        self.round_graph = False

    def _ensure_round_graph(self, share):
        """Capture the whole-round graph (one per round form: with / without the E-share) on first use; a capture
        the stack refuses (an RCCL or HIP build without collective capture) turns the whole-round graph off and the
        round takes the split path."""
        if share not in self._rgraph:
            try:
                self._rgraph[share] = self._capture_round(share)
            except RuntimeError as e:     # (a capture error leaves no work queued: nothing was issued)
                import warnings
                warnings.warn(f"whole-round graph capture failed, split rounds from now on: {e}")
                self.round_graph = False
                return False
        return True

    def _capture_round(self, share=False):
        s = self.step
        s._packed_current()
        g = torch.cuda.CUDAGraph()
        # thread-local capture mode: another thread's CUDA call (RCCL's watchdog polling its events) must not
        # invalidate this capture
        with torch.cuda.graph(g, capture_error_mode="thread_local"):   # (captures only: the caller replays it)
            s.run(C.PHASE_A, graph=False)
            self.exchange_mid()
            if share and self.d_side:   # the E-share of D on a side stream beside phase B
                main = torch.cuda.current_stream()
                side = self._side_stream()
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    self._d_exchange(-1, True, False)
                s.run(C.PHASE_B, graph=False)
                main.wait_stream(side)
            else:
                s.run(C.PHASE_B, graph=False)
                if share:
                    self._d_exchange(-1, True, False)
        return g

    def _d_exchange(self, r, share, swap):
        s = self.step
        if share:
            self.comm.all_reduce_mean(s.d_params)
        if swap:
            self.comm.swap([s.d_params], self.dswap.next_perm())
        if (share or swap) and hasattr(s, "sync_params_d"):
            s.sync_params_d()        # D's packed copies from the exchanged parameters (same stream)

    def _side_stream(self):
        if not self.step.d_params.is_cuda:
            return None
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(device=self.step.d_params.device)
        return self._side

    def cloud_average(self):
        """Data-size-weighted average of the shared trunk (+ its BatchNorm running stats) across
        server groups, mixed-gan.py:104-124 (weights A_s = data_len_s / sum).  With
        ``fedavg_compat_noop`` the reference's actual behaviour is reproduced: its load_state_dict
        ignores every key, so the Cloud is only a barrier."""
        if self.fedavg_compat_noop:
            self.cloud.all_reduce_sum(torch.zeros(1, device=self.step.g_params.device))
            return
        if self.cloud_scope == "trunk":
            p, r = self.step.trunk_slices()
        else:
            p, r = self.step.g_params, None
        for t in (p, r):
            if t is None:
                continue
            own = t.clone() if self.segema != 0.0 else None
            self.cloud.all_reduce_mean(t, self.cloud_weights)
            if own is not None:     # segema * self_p + (1 - segema) * recv_p, in that order
                torch.add(own * self.segema, t * (1.0 - self.segema), out=t)
        if hasattr(self.step, "sync_params"):
            self.step.sync_params()     # G's parameters changed outside the round: refresh its packed copies


def mixg_cloud_due(num_communication: int, cloud_epoch: int):
    """mixed-gan.py:193: the Cloud step runs before round r when t = num_communication - r satisfies
    ``cloud_epoch != 0 and t % cloud_epoch == 0``."""
    return lambda r: cloud_epoch != 0 and (num_communication - r) % cloud_epoch == 0


def capgan_cloud_due(num_communication: int, data_len: float, cloud_epoch: int, batch_size: int):
    """capgan.py:169: ``t % (self.data_len * cloud_epoch / batch_size) == 0`` with data_len the float32
    tensor sum of the shard sizes (Server.run :152) -- evaluated in the same float32 arithmetic, so a
    period that is not an integer never fires, as in the reference."""
    period = torch.tensor(float(data_len), dtype=torch.float32) * cloud_epoch / batch_size
    return lambda r: bool(torch.remainder(torch.tensor(float(num_communication - r), dtype=torch.float32),
                                          period) == 0)


class LocalComm:
    """N in-process workers in lockstep: the collectives of ``WorkerExchange`` computed over the
    workers' buffers with a fixed summation order (rank 0 .. N-1) -- the single-GPU rehearsal of a
    server group.  ``share_every``: E-share of D (a19); ``swap_every``: the MD-GAN D-swap
    with the server's ``DSwap`` permutation (MDGAN/MNIST/mdgan.py:158-164), moving the D parameters
    only, as ``WorkerExchange`` does (each worker keeps its own Adam state)."""

    def __init__(self, steps, share_every: int = 0, swap_every: int = 0, server_rank: int = 0):
        self.steps = steps
        self.size = len(steps)
        self.share_every, self.swap_every = share_every, swap_every
        self.dswap = DSwap(self.size, server_rank) if swap_every > 0 else None
        for s in steps:
            if s.n_workers != self.size:
                raise ValueError(f"step planned for {s.n_workers} workers, group has {self.size}")
            if self.size > 1 and hasattr(s, "set_exchange"):
                s.set_exchange("reduce")      # (this rehearsal runs alpha_scale + the summed exchange buffer)

    def round(self, r: int, graph: bool = False, share_every: int = None):
        ss = self.steps
        share_every = self.share_every if share_every is None else share_every
        if self.size == 1:
            ss[0].run(C.PHASE_ALL, graph=graph)
        else:
            for s in ss:
                s.run(C.PHASE_A, graph=graph)
            losses = torch.cat([s.own_loss() for s in ss])
            for s in ss:
                s.losses_all.copy_(losses)
                s.alpha_scale()
            bufs = [s.exchange_buffer() for s in ss]
            tot = bufs[0].clone()
            for b in bufs[1:]:
                tot += b
            for b in bufs:
                b.copy_(tot)
            for s in ss:
                s.run(C.PHASE_B, graph=graph)
        if share_every > 0 and (r + 1) % share_every == 0:
            tot = ss[0].d_params.clone()
            for s in ss[1:]:
                tot += s.d_params
            tot /= self.size
            for s in ss:
                s.d_params.copy_(tot)
        if self.dswap is not None and (r + 1) % self.swap_every == 0:
            perm = self.dswap.next_perm()
            old = [s.d_params.clone() for s in ss]
            for i, s in enumerate(ss):      # worker i continues with D_{perm[i]}
                s.d_params.copy_(old[perm[i]])
            return perm
        return None


def local_cloud_average(steps, weights, cloud_scope: str = "trunk", segema: float = 0.0,
                        fedavg_compat_noop: bool = False):
    """``WorkerExchange.cloud_average`` over in-process workers (the cloud group = ``steps``, one
    weight per member, e.g. A_s / group size for every replica of server s's trunk): every member
    ends with sum_i w_i t_i (fixed order 0 .. n-1), mixed with segema as mixed-gan.py:198-199."""
    if fedavg_compat_noop:
        return
    if len(weights) != len(steps):
        raise ValueError("one cloud weight per member")
    parts = [s.trunk_slices() if cloud_scope == "trunk" else (s.g_params, None) for s in steps]
    for which in (0, 1):
        ts = [p[which] for p in parts]
        if ts[0] is None:
            continue
        tot = ts[0] * float(weights[0])
        for w, t in zip(weights[1:], ts[1:]):
            tot += t * float(w)
        for t in ts:
            if segema != 0.0:
                torch.add(t * segema, tot * (1.0 - segema), out=t)
            else:
                t.copy_(tot)
    for s in steps:
        if hasattr(s, "sync_params"):
            s.sync_params()


class ConvWorkerExchange:
    """The same round for the conv GAN (cglgan.conv_step.ConvGanStep, model/lsgan.py): the exchange
    tensor is the image gradient dl/dXg [B, 32, 32, 1]; E-share averages D's parameters and its
    BatchNorm running statistics; D-swap moves both (the reference's copy_parameters keeps every
    non-scalar state-dict entry, MDGAN/MNIST/mdgan.py:233-238)."""

    def __init__(self, step, comm=None, share_every: int = 0, swap_every: int = 0, server_rank: int = 0,
                 force_split: bool = False):
        self.step, self.comm = step, comm
        self.share_every, self.swap_every = share_every, swap_every
        # test hook (as WorkerExchange's): the N > 1 path in a one-rank group, so a one-GPU box runs the
        # conv exchange over real RCCL
        self.force_split = force_split
        n = comm.size if comm is not None else 1
        if n != step.n_workers:
            raise ValueError(f"step planned for {step.n_workers} workers, group has {n}")
        # the server's own generator, Random(server_rank + 100) (MDGAN/MNIST/mdgan.py:122-123), as WorkerExchange
        self.dswap = DSwap(n, server_rank) if (comm is not None and swap_every > 0) else None

    def _d_state(self):
        return [self.step.D.p] + list(self.step.D.running.values())

    def rounds(self, r0: int, n: int):
        """Rounds r0 .. r0 + n - 1; with no group (N = 1) as multi-round graphs (ConvGanStep.run_rounds)."""
        if self.comm is None:
            self.step.run_rounds(n)
            return
        for r in range(r0, r0 + n):
            self.round(r)

    def round(self, r: int, real=None, eager=False):
        """One round.  N > 1: phase A, the exchange, phase B -- with a ConvGanStep(graph=True) drawing its
        own real batches, phase A and phase B replay as hipGraphs from the second round on
        (ConvGanStep.round_a / round_b); ``eager`` issues them op by op."""
        from . import conv_ops as O
        s = self.step
        share = self.comm is not None and self.share_every > 0 and (r + 1) % self.share_every == 0
        swap = self.dswap is not None and (r + 1) % self.swap_every == 0
        if self.comm is None or (self.comm.size == 1 and not self.force_split):
            s.run(real, eager=eager)
        else:
            s.round_a(real, eager=eager)
            self.comm.all_gather(s.losses_all, s.lbuf[2:3])
            O.weights_scale(s.weighting, s.lam, s.beta, s.losses_all, s.rank, s.dimg)
            self.comm.all_reduce_sum(s.dimg)
            if (share or swap) and s.D.p.is_cuda:
                # as WorkerExchange.round: phase B (G backward + Adam G) never touches D, so the D
                # exchange of this round runs on a side stream beside it, joined before the next round
                if getattr(self, "_side", None) is None:
                    self._side = torch.cuda.Stream(device=s.D.p.device)
                main = torch.cuda.current_stream()
                self._side.wait_stream(main)
                with torch.cuda.stream(self._side):
                    self._d_exchange(share, swap)
                s.round_b()
                main.wait_stream(self._side)
                share = swap = False
            else:
                s.round_b()
        self._d_exchange(share, swap)

    def _d_exchange(self, share, swap):
        if share:
            for t in self._d_state():
                self.comm.all_reduce_mean(t)
        if swap:
            self.comm.swap(self._d_state(), self.dswap.next_perm())


class ConvLocalComm:
    """N conv-GAN workers (cglgan.conv_step.ConvGanStep) of one process in lockstep -- the single-GPU
    rehearsal of ConvWorkerExchange: the same phase A / all-gather / alpha / sum / phase B sequence,
    the sums taken over the workers' buffers in a fixed order (rank 0 .. N-1)."""

    def __init__(self, steps):
        self.steps = steps
        self.size = len(steps)

    def round(self, r: int, reals=None, share_every: int = 0, eager=False):
        from . import conv_ops as O
        ss = self.steps
        reals = reals if reals is not None else [None] * self.size
        if self.size == 1:
            ss[0].run(reals[0], eager=eager)
            return
        for s, x in zip(ss, reals):
            s.round_a(x, eager=eager)
        losses = torch.cat([s.lbuf[2:3] for s in ss])
        for s in ss:
            s.losses_all.copy_(losses)
            O.weights_scale(s.weighting, s.lam, s.beta, s.losses_all, s.rank, s.dimg)
        tot = ss[0].dimg.clone()
        for s in ss[1:]:
            tot += s.dimg
        for s in ss:
            s.dimg.copy_(tot)
            s.round_b()
        if share_every > 0 and (r + 1) % share_every == 0:
            for i in range(1 + len(ss[0].D.running)):
                ts = [s.D.p if i == 0 else list(s.D.running.values())[i - 1] for s in ss]
                tot = ts[0].clone()
                for t in ts[1:]:
                    tot += t
                tot /= self.size
                for t in ts:
                    t.copy_(tot)
