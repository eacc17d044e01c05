"""The reference drivers' API on one process per MI355X.

The reference configures a run with module-level globals (capgan.py:26-58) plus two flags of
mixed-gan.py (``-c/--cloud_epoch``, ``-s/--segema``, :24-28), builds ``num_workers`` Worker threads
(D + shard), ``num_servers`` Server threads (G, lambda) and one Cloud thread, and assigns workers to
servers in consecutive blocks of ``num_workers // num_servers`` (capgan.py:509-516).  Here:

  * the same knobs, with the same names and defaults, are module globals of this module (set them
    before ``DriverConfig.from_module()``, as a reference user edits the globals) and CLI flags;
  * a Worker is a process on its own GPU (rank r of ``num_workers``); the Server role of server s is
    replicated on every worker of its block (G, lambda and Adam G are identical there: same init,
    same z stream, deterministic kernels), so the Server <-> Worker queues become collectives of the
    server group ``dist.new_group(block s)``;
  * the Cloud is the world group: its FedAvg (mixed-gan.py:104-124, 193-200; capgan.py:99-117,
    169-175) is a weighted all-reduce with weight A_s / H on each of server s's H replicas.

Algorithms (``algo``):
  ``capgan``  capgan.py:211-262 + :316-349 -- model/mnist_model.py G / D, CE, lambda-weighted
              alpha = softmax(softmax(lambda l) beta), Cloud = fedlab fedavg_aggregate of every G
              parameter before rounds with t % (data_len cloud_epoch / batch_size) == 0 (:169).
  ``mixg``    mixed-gan.py:238-292 + :355-392 -- MixGenerator (one head per worker of the server),
              trunk gradient exchanged inside the server group, alpha = softmax(beta lambda l)
              (``weighting="mix_double"``: CAPGAN/MNIST/mixed-gan.py:276-278), Cloud = A_s-weighted
              trunk average before rounds with t % cloud_epoch == 0 (:193).
  ``mdgan``   MDGAN/MNIST/mdgan.py:180-207 + :266-297 -- Sigmoid D, BCE, G on mean(l_i); optional
              D-swap every ``swap_every`` rounds (:158-164, commented out in the reference).
  E-share of D every ``share_every`` rounds (new behaviour) for any algorithm.

Data: there is no MNIST on these hosts (and the reference downloads it at import, capgan.py:57), so
the dataset is ``cglgan.data.synthetic_mnist`` (labelled, MNIST-shaped); the shards are the
reference's ``allocate_dataset(iid)`` cut of it (cglgan.data, pinned against the reference), resident
in HBM and sampled on device each round (DataLoader(shuffle=True) order: each pass over a shard ends
with its short batch of len(shard) mod batch_size rows, capgan.py:282, 326-331).

Usage (one process per GPU; ``torchrun`` sets RANK / WORLD_SIZE):
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 -m cglgan.driver \\
        --algo mixg --num_workers 8 --num_servers 2 --batch_size 256 -c 1 -s 0
"""
from __future__ import annotations

import argparse
import json
import os
import time
from dataclasses import asdict, dataclass, fields

import torch
import torch.distributed as dist

# ---- the reference's module-level knobs (capgan.py:26-58; mixed-gan.py:26-27 for -c / -s)
seed = 20211212
num_communication = 20000
cloud_epoch = 1
segema = 0.0
num_workers = 10
num_servers = 1
num_class = 10          # must be >= num_workers for iid 2 (capgan.py:44)
num_sample = 1000
iid = 0
batch_size = 100
frac_workers = 1        # the reference defines it and never reads it (capgan.py:49)
epoch = 1
b1 = 0.5
b2 = 0.999
img_size = 28
lr_g = 0.0002           # Server / Worker constructor defaults (capgan.py:122, 267)
lr_d = 0.0002

ALGOS = ("capgan", "mixg", "mdgan")
_DEFAULT_WEIGHTING = {"capgan": "capgan", "mixg": "mix_single", "mdgan": "mean"}


@dataclass
class DriverConfig:
    algo: str = "capgan"
    num_workers: int = 10
    num_servers: int = 1
    epoch: int = 1
    batch_size: int = 100
    num_communication: int = 20000
    cloud_epoch: int = 1
    segema: float = 0.0
    iid: int = 0
    num_class: int = 10
    num_sample: int = 1000
    b1: float = 0.5
    b2: float = 0.999
    lr_g: float = 0.0002
    lr_d: float = 0.0002
    seed: int = 20211212
    img_size: int = 28
    # build-side knobs (not in the reference)
    weighting: str = ""              # "" = the algorithm's own; "mix_double" for CAPGAN/MNIST/mixed-gan.py
    share_every: int = 0             # E-share of D every E rounds (a19); 0 = off
    swap_every: int = 0              # MD-GAN D-swap every E rounds; 0 = off
    fedavg_compat_noop: bool = False  # reproduce the reference's no-op Cloud load
    dataset_rows: int = 60000        # synthetic MNIST-shaped dataset (MNIST's train size)
    data_seed: int = 11
    log_every: int = 0
    checkpoint_dir: str = ""
    resume_dir: str = ""             # per-worker resume files (new): written every resume_every rounds
    resume_every: int = 0            #   and at the end; a run started with an existing file resumes
    graph: bool = True
    gemm_dtype: str = "f32"          # "f16" / "bf16": 16-bit GEMM operands (BASELINE config 5's fp16)
    loss_scale: float = 0.0          # dynamic loss scaling of the 16-bit path (initial scale; 0 = off)

    @classmethod
    def from_module(cls, **overrides):
        """The module globals above (as the reference reads its own), then ``overrides``."""
        g = globals()
        kw = {f.name: g[f.name] for f in fields(cls) if f.name in g}
        kw.update(overrides)
        return cls(**kw)

    def validate(self):
        if self.algo not in ALGOS:
            raise ValueError(f"algo must be one of {ALGOS}")
        if self.num_servers < 1 or self.num_workers % self.num_servers:
            raise ValueError("num_workers must be a positive multiple of num_servers (capgan.py:509-516 drops "
                             "the remainder workers; here every GPU is a worker)")
        if self.algo == "mdgan" and self.num_servers != 1:
            raise ValueError("MD-GAN has one server (MDGAN/MNIST/mdgan.py)")
        if self.iid == 2 and self.num_class < self.num_workers:
            raise ValueError("iid 2 needs num_class >= num_workers (capgan.py:44)")
        if self.epoch < 1 or self.batch_size < 2:
            raise ValueError("epoch >= 1 and batch_size >= 2 (train-mode BatchNorm)")
        return self

    @property
    def heads(self):
        return self.num_workers // self.num_servers

    @property
    def weighting_(self):
        return self.weighting or _DEFAULT_WEIGHTING[self.algo]


class Topology:
    """Server / worker assignment of capgan.py:509-516: server s serves workers
    [s H, (s + 1) H), H = num_workers // num_servers; rank r is worker r."""

    def __init__(self, num_workers: int, num_servers: int, rank: int):
        if num_workers % num_servers:
            raise ValueError("num_workers must be a multiple of num_servers")
        self.num_workers, self.num_servers = num_workers, num_servers
        self.heads = num_workers // num_servers
        self.rank = rank
        self.server = rank // self.heads
        self.local = rank % self.heads

    def members(self, s=None):
        s = self.server if s is None else s
        return list(range(s * self.heads, (s + 1) * self.heads))

    def make_groups(self):
        """Every rank creates every server group (dist.new_group is collective, same order on all
        ranks); returns this rank's server group (None when it is the whole world)."""
        if self.num_servers == 1:
            return None
        mine = None
        for s in range(self.num_servers):
            g = dist.new_group(self.members(s))
            if s == self.server:
                mine = g
        return mine


def make_shards(cfg: DriverConfig):
    """The synthetic dataset and the reference's allocate_dataset cut of it (identical on every rank:
    the driver's Random(seed) drives it, capgan.py:25-27)."""
    from .data import allocate_dataset, driver_rng, synthetic_mnist
    x, y = synthetic_mnist(cfg.dataset_rows, cfg.num_class, seed=cfg.data_seed, img_dim=cfg.img_size ** 2)
    _, shards, _ = allocate_dataset(y, cfg.iid, cfg.num_workers, cfg.num_class, cfg.num_sample,
                                    rd=driver_rng(cfg.seed))
    return x, shards


def gpu_step(cfg: DriverConfig, topo: Topology, shard: torch.Tensor, beta, g_sd, d_sd, device):
    """The fused HIP worker round (cglgan.GanStep) of this rank, loaded with the initial state."""
    from . import specs
    from .step import GanStep
    img = cfg.img_size ** 2
    gm, loss, xl = specs.mnist_generator(img), "ce", -1
    dm = specs.mnist_discriminator(img, sigmoid=(cfg.algo == "mdgan"))
    if cfg.algo == "mixg":
        gm, xl = specs.mixgen_worker(topo.local, img), specs.MIXGEN_HEAD_LAYER
    if cfg.algo == "mdgan":
        loss = "bce"
    # the whole shard: the in-graph sampler is DataLoader(shuffle=True) over it, each pass ending
    # with the short batch of len(shard) mod batch_size rows (capgan.py:282, 326-331)
    if shard.shape[0] == 0:
        raise ValueError(f"worker {topo.rank}: empty shard")
    real = shard.to(device=device, dtype=torch.float32).contiguous()
    step = GanStep(gm, dm, batch=cfg.batch_size, epoch=cfg.epoch, loss=loss, weighting=cfg.weighting_,
                   n_workers=topo.heads, rank=topo.local, exchange_layer=xl, lr_g=cfg.lr_g, lr_d=cfg.lr_d,
                   betas=(cfg.b1, cfg.b2), seed=cfg.seed + 7919 * topo.server, gen_z=True, real=real,
                   sample_n=real.shape[0], device=device, gemm_dtype=cfg.gemm_dtype,
                   loss_scale=cfg.loss_scale)
    step.load_state_dicts(g_sd, d_sd)
    step.reset(beta=beta)
    return step


def capgan_cloud_schedule(cfg: DriverConfig, srv_lens, server: int):
    """The Cloud schedule of a multi-server CAPGAN run (capgan.py:169, Cloud.run :99-117).

    Each reference server syncs before rounds with t % (data_len * cloud_epoch / batch_size) == 0,
    data_len = ITS OWN shard total, and the Cloud averages whichever ``num_servers`` puts arrive
    next.  Servers with different shard totals therefore sync on different rounds and a different
    number of times: the Cloud pairs one server's puts with each other (``p[idx]`` overwritten) and a
    server blocks forever on its cache -- the reference hangs.  Here every Cloud step is a world
    all-reduce, so all servers must fire on the same rounds: the schedule is used when every
    server's period gives the same set of rounds over the run, and such a run is refused otherwise
    (equal-size servers -- iid 0 -- or ``cloud_epoch = 0`` keep it well defined)."""
    from .exchange import capgan_cloud_due
    dues = [capgan_cloud_due(cfg.num_communication, float(n), cfg.cloud_epoch, cfg.batch_size) for n in srv_lens]
    if len(set(srv_lens)) > 1:
        fire = [[r for r in range(cfg.num_communication) if d(r)] for d in dues]
        if any(f != fire[0] for f in fire[1:]):
            raise ValueError(
                "capgan with num_servers > 1: the servers' Cloud periods t % (data_len * cloud_epoch / batch_size) "
                f"differ (server shard totals {list(srv_lens)}); the reference Cloud deadlocks on such a run "
                "(capgan.py:108-117, :169-175). Use equal-size servers (iid 0), cloud_epoch 0, or algo mixg.")
    return dues[server]


class Driver:
    """One worker process of a CAPGAN / Mix-G / MD-GAN run (see module docstring)."""

    def __init__(self, cfg: DriverConfig, rank: int = None, world: int = None, step_factory=None, device=None):
        from .data import beta_weights, cloud_weights
        from .exchange import DistComm, WorkerExchange, mixg_cloud_due
        from .init import topology_state
        self.cfg = cfg.validate()
        dist_on = dist.is_available() and dist.is_initialized()
        self.rank = rank if rank is not None else (dist.get_rank() if dist_on else 0)
        self.world = world if world is not None else (dist.get_world_size() if dist_on else 1)
        if self.world != cfg.num_workers:
            raise ValueError(f"one process per worker: world size {self.world} != num_workers {cfg.num_workers}")
        self.topo = topo = Topology(cfg.num_workers, cfg.num_servers, self.rank)
        group = topo.make_groups() if self.world > 1 else None
        x, shards = make_shards(cfg)
        lens = [len(s) for s in shards]
        self.beta, data_len = beta_weights([lens[i] for i in topo.members()])
        self.beta = self.beta.tolist()
        srv_lens = [sum(lens[i] for i in topo.members(s)) for s in range(cfg.num_servers)]
        A = cloud_weights(srv_lens).tolist()
        gs, ds = topology_state(cfg.algo, cfg.num_servers, cfg.num_workers, cfg.seed, cfg.img_size ** 2)
        shard = x[torch.as_tensor(shards[self.rank])]
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
        factory = step_factory or gpu_step
        self.step = factory(cfg, topo, shard, self.beta, gs[topo.server], ds[self.rank], device)
        comm = DistComm(group) if topo.heads > 1 else None
        cloud, due, scope = None, None, "trunk"
        if cfg.num_servers > 1 and cfg.cloud_epoch != 0:
            cloud = DistComm(None)
            if cfg.algo == "mixg":
                due = mixg_cloud_due(cfg.num_communication, cfg.cloud_epoch)
            else:
                due = capgan_cloud_schedule(cfg, srv_lens, topo.server)
                scope = "all"
        # one weight per member of the cloud group (the world): A_s / H on each replica of server s
        cw = [A[r // topo.heads] / topo.heads for r in range(self.world)]
        self.exchange = WorkerExchange(self.step, comm, share_every=cfg.share_every, cloud=cloud, cloud_weights=cw,
                                       fedavg_compat_noop=cfg.fedavg_compat_noop, swap_every=cfg.swap_every,
                                       cloud_scope=scope, segema=cfg.segema, cloud_due=due, server_rank=topo.server)
        self.lambda_list = []
        self.round = 0
        if cfg.resume_dir:
            err = None
            if os.path.exists(self.resume_path()):
                try:
                    self.load_resume()
                except Exception as e:        # raised on every rank together below, not here alone
                    err = e
            self._check_resumed_round(err)

    def run(self, rounds: int = None, log=print):
        """``rounds`` communication rounds (default: num_communication), as Server.run's
        ``while t > 0`` loop (capgan.py:164-196)."""
        cfg = self.cfg
        n = cfg.num_communication if rounds is None else rounds
        if rounds is None:
            n = max(0, n - self.round)          # a resumed run finishes the schedule it started
        t0 = time.perf_counter()
        for _ in range(n):
            self.exchange.round(self.round, graph=cfg.graph)
            self.round += 1
            if cfg.resume_dir and cfg.resume_every and self.round % cfg.resume_every == 0:
                self.save_resume()
            if cfg.log_every and self.round % cfg.log_every == 0:
                st = self.step.stats()
                self.lambda_list.append(st.get("lambda"))
                if self.topo.local == 0 and log is not None:
                    log(json.dumps({"round": self.round, "server": self.topo.server, "d_loss": st["d_loss"],
                                    "g_loss": st["g_loss"], "lambda": st.get("lambda"), "F": st.get("F"),
                                    "s": round(time.perf_counter() - t0, 3)}))
        if cfg.checkpoint_dir and self.topo.local == 0:
            self.save(cfg.checkpoint_dir)
        if cfg.resume_dir:
            self.save_resume()
        return self.step.stats()

    # ---------------------------------------------------------------- resume (new)
    def resume_path(self):
        return os.path.join(self.cfg.resume_dir, f"resume-{self.cfg.algo}-rank{self.rank}.pt")

    # every knob that changes the trajectory or the schedule of a run: a file saved under other settings
    # is refused instead of continuing a different run.  num_communication is one of them on purpose: the
    # Mix-G Cloud schedule (mixg_cloud_due) and the CAPGAN S > 1 schedule are cut from it, so a resumed run
    # with a larger round budget would not continue the run that was saved -- extending a run is refused.
    RESUME_KEYS = ("algo", "num_workers", "num_servers", "epoch", "batch_size", "num_communication", "cloud_epoch",
                   "segema", "iid", "num_class", "num_sample", "b1", "b2", "lr_g", "lr_d", "seed", "img_size",
                   "weighting", "share_every", "swap_every", "fedavg_compat_noop", "dataset_rows", "data_seed",
                   "gemm_dtype", "loss_scale")

    def _resume_key(self):
        c = self.cfg
        return json.dumps({k: getattr(c, k) for k in self.RESUME_KEYS}, sort_keys=True)

    def _rng_states(self):
        """The exchange's host-side generators (the MD-GAN D-swap's Random(server + 100)) as plain lists
        (weights_only-loadable): a resumed run draws the permutations the uninterrupted run would."""
        ds = getattr(self.exchange, "dswap", None)
        if ds is None:
            return None
        ver, ints, gauss = ds.rd.getstate()
        return [int(ver), [int(x) for x in ints], gauss]

    def save_resume(self):
        from .checkpoint import save_resume
        return save_resume(self.step, self.resume_path(), round=self.round, rank=self.rank,
                           config=self._resume_key(), lambda_list=[float(x) for x in self.lambda_list if x is not None],
                           dswap_state=self._rng_states())

    def load_resume(self):
        from .checkpoint import load_resume
        meta = load_resume(self.step, self.resume_path())
        if meta.get("config") != self._resume_key() or meta.get("rank") != self.rank:
            raise ValueError(f"{self.resume_path()}: saved by a different configuration or rank")
        self.round = int(meta["round"])
        self.lambda_list = list(meta.get("lambda_list", []))
        ds = getattr(self.exchange, "dswap", None)
        saved = meta.get("dswap_state")
        if (ds is None) != (saved is None):
            raise ValueError(f"{self.resume_path()}: D-swap generator state does not match this run")
        if ds is not None:
            ds.rd.setstate((int(saved[0]), tuple(int(x) for x in saved[1]), saved[2]))

    def _check_resumed_round(self, err=None):
        """Every rank must continue from the same round (a crash between two ranks' file replacements
        leaves files of different rounds; the collectives would then pair different rounds or hang):
        min and max of the resumed round over the world must agree.  A rank whose own load failed
        (``err``) joins the same all-reduce with its error flag raised, so every rank raises together
        instead of the others waiting in a collective until the process-group timeout."""
        if self.world == 1 or not (dist.is_available() and dist.is_initialized()):
            if err is not None:
                raise err
            return
        dev = self.step.g_params.device if dist.get_backend() == "nccl" else torch.device("cpu")
        t = torch.tensor([1 if err is not None else 0, self.round, -self.round], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        bad, hi, lo = int(t[0]), int(t[1]), -int(t[2])
        if err is not None:
            raise err
        if bad:
            raise RuntimeError(f"rank {self.rank}: another rank failed to load its resume file in "
                               f"{self.cfg.resume_dir}")
        if hi != lo:
            raise RuntimeError(f"rank {self.rank}: resume files of different rounds across the world "
                               f"(min {lo}, max {hi}) in {self.cfg.resume_dir}")

    def save(self, directory):
        """capgan.py:185-200: the server's generator state dict + its config pickle."""
        from .checkpoint import save_server
        name = f"{self.cfg.algo}-server{self.topo.server}-iid{self.cfg.iid}-epoch{self.cfg.epoch}"
        return save_server(self.step, directory, name, self.topo.members(), self.beta, self.lambda_list)


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    d = DriverConfig.from_module()
    p.add_argument("--algo", choices=ALGOS, default=d.algo)
    p.add_argument("-c", "--cloud_epoch", default=d.cloud_epoch, type=int)        # mixed-gan.py:26
    p.add_argument("-s", "--segema", default=d.segema, type=float)                # mixed-gan.py:27
    for name in ("num_workers", "num_servers", "epoch", "batch_size", "num_communication", "iid", "num_class",
                 "num_sample", "seed", "img_size", "share_every", "swap_every", "dataset_rows", "data_seed",
                 "log_every"):
        p.add_argument(f"--{name}", type=int, default=getattr(d, name))
    for name in ("b1", "b2", "lr_g", "lr_d"):
        p.add_argument(f"--{name}", type=float, default=getattr(d, name))
    p.add_argument("--weighting", default="", choices=["", "capgan", "mean", "mix_single", "mix_double"])
    p.add_argument("--fedavg_compat_noop", action="store_true")
    p.add_argument("--checkpoint_dir", default="")
    p.add_argument("--resume_dir", default="", help="per-worker resume files (written; resumed from if present)")
    p.add_argument("--resume_every", type=int, default=0)
    p.add_argument("--eager", action="store_true", help="launch the round without hipGraph replay")
    p.add_argument("--gemm_dtype", default="f32", choices=["f32", "f16", "bf16"],
                   help="GEMM operand type (f16 / bf16: 16-bit operands, fp32 accumulation; BASELINE config 5)")
    p.add_argument("--loss_scale", type=float, default=0.0,
                   help="16-bit path: dynamic loss scaling from this initial scale (power of two, e.g. 65536)")
    return p.parse_args(argv)


def main(argv=None):
    a = parse_args(argv)
    kw = {f.name: getattr(a, f.name) for f in fields(DriverConfig) if hasattr(a, f.name)}
    kw["graph"] = not a.eager
    cfg = DriverConfig(**kw)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
    if world > 1 and not dist.is_initialized():
        if torch.cuda.is_available():
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    try:
        drv = Driver(cfg)
        if drv.rank == 0:
            print(json.dumps({"config": asdict(cfg), "world": drv.world,
                              "backend": dist.get_backend() if dist.is_initialized() else None}), flush=True)
        st = drv.run()
        if drv.topo.local == 0:
            print(json.dumps({"final": True, "server": drv.topo.server, "round": st["round"],
                              "d_loss": st["d_loss"], "g_loss": st["g_loss"]}), flush=True)
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


if __name__ == "__main__":
    main()
