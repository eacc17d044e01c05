"""One worker's fused GAN round on its own MI355X: the drop-in for the reference's
Server.train + Worker.train pair (capgan.py:211-262 + :316-349, mixed-gan.py:238-292 + :355-392,
MDGAN/MNIST/mdgan.py:180-207 + :266-297, CGLGAN/2DMG/main.py:225-278 + :344-375).

All device memory is allocated here with torch (the caching allocator owns it); the HIP library
borrows it.  Parameters live in one flat fp32 buffer per model (G, D) with the reference's
state-dict keys exposed as views, so ``state_dict()`` / ``load_state_dict()`` interoperate with
checkpoints written by the reference (``torch.save(net_g.state_dict())`` capgan.py:186).
"""
from __future__ import annotations

import ctypes
from collections import OrderedDict

import torch

from . import _lib as C
from .specs import MlpModel

_WEIGHTING = {"capgan": C.WEIGHT_CAPGAN, "mean": C.WEIGHT_MEAN, "mix_single": C.WEIGHT_MIX_SINGLE,
              "mix_double": C.WEIGHT_MIX_DOUBLE, "cglgan": C.WEIGHT_CGLGAN}


def _spec(m: MlpModel) -> C.MlpSpec:
    s = C.MlpSpec()
    s.n_layers = m.n_layers
    for i, v in enumerate(m.dims):
        s.dims[i] = v
    for i, v in enumerate(m.bn):
        s.bn[i] = v
    return s


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


_DTYPE = {"f32": C.DTYPE_F32, "f16": C.DTYPE_F16, "bf16": C.DTYPE_BF16}


class GanStep:
    """Fused worker round.  ``run()`` = one communication round of one worker.

    Knobs mirror the reference drivers' module globals: ``batch`` (batch_size, capgan.py:48),
    ``epoch`` (local D steps, capgan.py:50), ``b1``/``b2`` (capgan.py:52-53), lr 2e-4 (:122).

    Packed weight copies: the GEMMs read fragment-packed copies of G's and D's weight matrices, kept current by
    the rounds' own Adam launches.  A write of ``g_params`` / ``d_params`` (or of any view of them) from outside the
    round is noticed through torch's version counter and the copies are refreshed before the next round.  Writes the
    counter does not see -- through ``.data``, DLPack or another library, or an in-place collective issued by the
    caller on the raw buffer -- must be followed by ``sync_params()`` (both models) or ``sync_params_d()`` (D only);
    otherwise the next rounds run on the old weights.  (G's copies are re-packed inside every round by the forward
    BatchNorm / loss-head launches; D's copies and the next round's z are the ones a missed write leaves stale.)
    """

    def __init__(self, g: MlpModel, d: MlpModel, batch: int, batch_real: int = None, epoch: int = 1,
                 loss: str = "ce", weighting: str = "capgan", n_workers: int = 1, rank: int = 0,
                 exchange_layer: int = -1, lr_g: float = 2e-4, lr_d: float = 2e-4, betas=(0.5, 0.999),
                 adam_eps: float = 1e-8, bn_eps: float = 0.8, bn_momentum: float = 0.1, slope: float = 0.2,
                 seed: int = 20211212, gen_z: bool = False, real: torch.Tensor = None, sample_n: int = 0,
                 real_idx: torch.Tensor = None, device="cuda", gemm_dtype: str = "f32", loss_scale: float = 0.0,
                 scale_growth_interval: int = 2000):
        """``gemm_dtype``: "f32" (the reference arithmetic), or "f16" / "bf16": every GEMM operand
        rounded to 16 bits at the matrix core with fp32 accumulation (BASELINE config 5's fp16;
        fp32 master weights, BatchNorm, losses and Adam; outside the fp32 parity band).
        ``loss_scale`` > 0 (16-bit only, a power of two; torch's GradScaler default is 65536): dynamic
        loss scaling with torch.cuda.amp.GradScaler semantics, one scaler per model -- the loss
        gradient enters the backward pass multiplied by the scale, the weight gradients are unscaled
        before Adam, a round whose gradients hold an inf / NaN skips that model's Adam step and halves
        its scale, ``scale_growth_interval`` clean rounds double it (include/cglgan.h)."""
        self.gm, self.dm = g, d
        self.B = batch
        self.Br = batch_real or batch
        self.epoch = epoch
        self.device = torch.device(device)
        cfg = C.GanConfig()
        cfg.g, cfg.d = _spec(g), _spec(d)
        cfg.batch, cfg.batch_real, cfg.epoch = batch, self.Br, epoch
        cfg.loss = C.LOSS_CE2 if loss == "ce" else C.LOSS_BCE
        cfg.weighting = _WEIGHTING[weighting]
        cfg.n_workers, cfg.rank, cfg.exchange_layer = n_workers, rank, exchange_layer
        cfg.lr_g, cfg.lr_d = lr_g, lr_d
        cfg.beta1, cfg.beta2, cfg.adam_eps = betas[0], betas[1], adam_eps
        cfg.bn_eps, cfg.bn_momentum, cfg.slope = bn_eps, bn_momentum, slope
        cfg.seed, cfg.gen_z, cfg.sample_n = seed, int(gen_z), sample_n
        if gemm_dtype not in _DTYPE:
            raise ValueError(f"gemm_dtype must be one of {sorted(_DTYPE)}")
        cfg.gemm_dtype = _DTYPE[gemm_dtype]
        self.gemm_dtype = gemm_dtype
        if loss_scale and gemm_dtype == "f32":
            raise ValueError("loss_scale applies to the 16-bit GEMM paths (gemm_dtype f16 / bf16)")
        cfg.loss_scale, cfg.scale_growth_interval = float(loss_scale), int(scale_growth_interval)
        self.cfg = cfg
        self.n_workers, self.rank = n_workers, rank
        self.exchange_layer = exchange_layer

        dev = self.device
        f32 = dict(dtype=torch.float32, device=dev)
        ng = C.lib.cgl_gan_param_count(ctypes.byref(cfg), C.MODEL_G)
        nd = C.lib.cgl_gan_param_count(ctypes.byref(cfg), C.MODEL_D)
        nr = C.lib.cgl_gan_running_count(ctypes.byref(cfg))
        wsb = C.lib.cgl_gan_workspace_bytes(ctypes.byref(cfg))
        if ng < 0 or nd < 0 or wsb < 0:
            raise RuntimeError(f"invalid GAN configuration (rc={min(ng, nd, wsb)})")
        self.g_params, self.g_grads = torch.zeros(ng, **f32), torch.zeros(ng, **f32)
        self.g_m, self.g_v = torch.zeros(ng, **f32), torch.zeros(ng, **f32)
        self.g_running = torch.zeros(max(nr, 1), **f32)
        self.d_params, self.d_grads = torch.zeros(nd, **f32), torch.zeros(nd, **f32)
        self.d_m, self.d_v = torch.zeros(nd, **f32), torch.zeros(nd, **f32)
        self.z = torch.zeros(2 * batch, g.dims[0], **f32)
        img = g.dims[-1]
        if real is None:
            real = torch.zeros(epoch * self.Br, img, **f32)
        self.real = real
        self.real_idx = real_idx
        self.losses_all = torch.zeros(max(n_workers, 1), **f32)
        self.workspace = torch.zeros(wsb, dtype=torch.uint8, device=dev)

        bufs = C.GanBuffers()
        for name in ("g_params", "g_grads", "g_m", "g_v", "g_running", "d_params", "d_grads", "d_m", "d_v", "z",
                     "real", "losses_all", "workspace"):
            setattr(bufs, name, self.__dict__[name].data_ptr())
        bufs.real_idx = real_idx.data_ptr() if real_idx is not None else None
        bufs.workspace_bytes = wsb
        self._bufs = bufs
        h = ctypes.c_void_p()
        C.check(C.lib.cgl_gan_create(ctypes.byref(cfg), ctypes.byref(bufs), ctypes.byref(h)), "cgl_gan_create")
        self._h = h
        self._pk_ver = None        # the packed weight copies (G, D): refreshed before the first round (sync_params)
        self.g_views = self._views(g, C.MODEL_G, self.g_params)
        self.d_views = self._views(d, C.MODEL_D, self.d_params)
        self.g_grad_views = self._views(g, C.MODEL_G, self.g_grads)
        self.d_grad_views = self._views(d, C.MODEL_D, self.d_grads)
        self._running_views()
        self.reset()

    # ------------------------------------------------------------------ layout views
    def _views(self, m: MlpModel, which, flat):
        keys = m.tensor_keys()
        out = OrderedDict()
        for i, k in enumerate(keys):
            off, rows, cols, layer, kind = (ctypes.c_int64(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int(),
                                            ctypes.c_int())
            C.check(C.lib.cgl_gan_param_tensor(ctypes.byref(self.cfg), which, i, ctypes.byref(off), ctypes.byref(rows),
                                               ctypes.byref(cols), ctypes.byref(layer), ctypes.byref(kind)))
            n = rows.value * cols.value
            v = flat[off.value:off.value + n]
            out[k] = v.view(rows.value, cols.value) if kind.value == 0 else v
        return out

    def trunk_slices(self):
        """(flat G-parameter view, flat running-stat view or None) of the layers below
        ``exchange_layer`` -- the Mix-G trunk shared by a server group (mixed-gan.py:193-200).
        Both are contiguous prefixes of the flat buffers (state-dict order)."""
        if self.exchange_layer <= 0:
            raise RuntimeError("no trunk: the step was planned without a trunk/head split")
        end = None
        for i in range(len(self.gm.tensor_keys())):
            off, rows, cols, layer, kind = (ctypes.c_int64(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int(),
                                            ctypes.c_int())
            C.check(C.lib.cgl_gan_param_tensor(ctypes.byref(self.cfg), C.MODEL_G, i, ctypes.byref(off),
                                               ctypes.byref(rows), ctypes.byref(cols), ctypes.byref(layer),
                                               ctypes.byref(kind)))
            if layer.value >= self.exchange_layer:
                end = off.value
                break
        p = self.g_params[:end]
        al = lambda n: (n + 63) // 64 * 64
        rend = sum(2 * al(self.gm.dims[l + 1]) for l in self.gm.bn_layers() if l < self.exchange_layer)
        return p, (self.g_running[:rend] if rend > 0 else None)

    def _running_views(self):
        self.running = OrderedDict()
        off = 0
        al = lambda n: (n + 63) // 64 * 64
        for l in self.gm.bn_layers():
            n = self.gm.dims[l + 1]
            k = self.gm.bn_keys[l]
            self.running[k + ".running_mean"] = self.g_running[off:off + n]
            off += al(n)
            self.running[k + ".running_var"] = self.g_running[off:off + n]
            off += al(n)

    # ------------------------------------------------------------------ state
    def reset(self, beta=None):
        """Zero lambda / round counters, set beta (data-size weights, capgan.py:149-153)."""
        b = beta if beta is not None else [1.0 / self.n_workers] * self.n_workers
        arr = (ctypes.c_float * len(b))(*[float(x) for x in b])
        C.check(C.lib.cgl_gan_reset(self._h, arr, _stream()), "cgl_gan_reset")
        self._pk_ver = self._pver()                  # (reset re-packs the weights)
        for k, v in self.running.items():
            v.fill_(0.0 if k.endswith("running_mean") else 1.0)

    @torch.no_grad()
    def load_state_dicts(self, g_sd, d_sd):
        for k, v in self.g_views.items():
            v.copy_(g_sd[k].reshape(v.shape))
        for k, v in self.d_views.items():
            v.copy_(d_sd[k].reshape(v.shape))
        for k, v in self.running.items():
            if k in g_sd:
                v.copy_(g_sd[k])
        self.g_m.zero_(); self.g_v.zero_(); self.d_m.zero_(); self.d_v.zero_()

    def g_state_dict(self):
        sd = OrderedDict()
        st = self.stats()
        for k, v in self.g_views.items():
            sd[k] = v.detach().clone()
        for l in self.gm.bn_layers():
            k = self.gm.bn_keys[l]
            sd[k + ".running_mean"] = self.running[k + ".running_mean"].clone()
            sd[k + ".running_var"] = self.running[k + ".running_var"].clone()
            sd[k + ".num_batches_tracked"] = torch.tensor(st["bn_batches"], dtype=torch.long)
        return sd

    def modules(self, img_shape=(1, 28, 28)):
        """(Generator, Discriminator) nn.Modules of cglgan.model holding a copy of this worker's
        current state (reference keys), e.g. for sampling G(fixed_z) in eval mode
        (capgan.py:203-209) or for checkpointing as the reference does."""
        from . import model as M
        if self.gm.name != "mnist_generator" or not self.dm.name.startswith("mnist_discriminator"):
            raise NotImplementedError("module export is provided for the model/mnist_model.py G / D")
        g = M.Generator(img_shape).to(self.device)
        d = M.Discriminator(img_shape, sigmoid=self.dm.name.endswith("sigmoid")).to(self.device)
        g.load_state_dict(self.g_state_dict())
        d.load_state_dict(self.d_state_dict())
        return g, d

    def d_state_dict(self):
        return OrderedDict((k, v.detach().clone()) for k, v in self.d_views.items())

    # ------------------------------------------------------------------ resume
    _RESUME_BUFS = ("g_params", "g_m", "g_v", "g_running", "d_params", "d_m", "d_v")

    def resume_state(self):
        """Everything the next round reads (SURVEY 5 "resume"): G / D parameters, both Adams' moments,
        the BatchNorm running statistics and the device round state (round counter -- which also
        drives the z stream, the sampler position and the Adam step counts --, lambda, beta),
        as CPU tensors.  The reference only saves the generator (capgan.py:185-200)."""
        torch.cuda.current_stream().synchronize()
        out = OrderedDict((k, getattr(self, k).detach().cpu().clone()) for k in self._RESUME_BUFS)
        out["device_state"] = self.internal(6).view(torch.int32).cpu().clone()
        return out

    @torch.no_grad()
    def load_resume_state(self, sd):
        for k in self._RESUME_BUFS:
            dst = getattr(self, k)
            if sd[k].shape != dst.shape:
                raise ValueError(f"resume state {k}: shape {tuple(sd[k].shape)} != {tuple(dst.shape)}")
            dst.copy_(sd[k])
        st = self.internal(6).view(torch.int32)
        if sd["device_state"].shape != st.shape:
            raise ValueError("resume state: device round state of another build / configuration")
        st.copy_(sd["device_state"])
        self.sync_params()          # the packed G weights and the next round's z from the loaded state
        torch.cuda.current_stream().synchronize()

    # ------------------------------------------------------------------ execution
    def sync_params(self):
        """Refresh the fragment-packed copies of G's weight matrices that its GEMMs read (cgl_gan_sync_params):
        the G Adam launch keeps them current, so this is needed only after G's parameters were written from
        outside the round (state-dict loads, init, the Cloud FedAvg).  Stream-ordered, no host sync."""
        C.check(C.lib.cgl_gan_sync_params(self._h, _stream()), "cgl_gan_sync_params")
        self._pk_ver = self._pver()

    def sync_params_d(self):
        """Refresh D's packed copies only (cgl_gan_sync_params_d): after D's parameters were written from outside the
        round by an E-share / D-swap.  Stream-ordered and capturable (the whole-round graph of a share round)."""
        C.check(C.lib.cgl_gan_sync_params_d(self._h, _stream()), "cgl_gan_sync_params_d")
        if self._pk_ver is not None:
            self._pk_ver = (self._pk_ver[0], self.d_params._version)

    def _pver(self):
        return (self.g_params._version, self.d_params._version)

    def _packed_current(self):
        # any in-place torch write of G's parameters (through g_params or one of its views) moves the buffer's
        # version counter; the library's own kernel writes do not, and they keep the packed copies current
        if self._pver() != self._pk_ver:
            self.sync_params()

    def run(self, phase=C.PHASE_ALL, graph=False):
        self._packed_current()
        fn = C.lib.cgl_gan_run_graph if graph else C.lib.cgl_gan_run
        C.check(fn(self._h, phase, _stream()), "cgl_gan_run")

    def run_rounds(self, rounds: int, graph: bool = True):
        """``rounds`` complete rounds (N = 1 or the caller's own lockstep): with ``graph`` one hipGraph launch holding
        them back to back (cgl_gan_run_graph_rounds: no graph-launch boundary between the rounds), else that many
        ``run()`` calls.  Identical to ``rounds`` calls of ``run(graph=graph)``."""
        if rounds <= 0:
            return
        if not graph:
            for _ in range(rounds):
                self.run(C.PHASE_ALL, graph=False)
            return
        self._packed_current()
        C.check(C.lib.cgl_gan_run_graph_rounds(self._h, int(rounds), _stream()), "cgl_gan_run_graph_rounds")

    def prepare_rounds(self, rounds: int):
        """Capture the ``rounds``-round graph ahead of its first use (one stream synchronisation)."""
        if rounds >= 2:
            C.check(C.lib.cgl_gan_prepare_graph_rounds(self._h, int(rounds), _stream()), "cgl_gan_prepare_graph_rounds")

    def alpha_scale(self):
        C.check(C.lib.cgl_gan_alpha_scale(self._h, _stream()), "cgl_gan_alpha_scale")

    exchange_mode = "reduce"

    def set_exchange(self, mode):
        """"reduce": the caller gathers the losses, calls alpha_scale and all-reduces exchange_buffer();
        "gather": the caller all-gathers gather_buffers()[0] into gather_buffers()[1] and phase B combines
        (include/cglgan.h cgl_gan_exchange_mode)."""
        C.check(C.lib.cgl_gan_exchange_mode(self._h, {"reduce": 0, "gather": 1}[mode]), "cgl_gan_exchange_mode")
        self.exchange_mode = mode

    def gather_buffers(self):
        """(send [slot], recv [n_workers * slot]): this worker's [exchange gradient | G loss | pad] slot, written
        by phase A, and the all-gather target phase B's combine reads."""
        if getattr(self, "_gbufs", None) is None:
            s, r, n = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_int64()
            C.check(C.lib.cgl_gan_gather_buffers(self._h, ctypes.byref(s), ctypes.byref(r), ctypes.byref(n)),
                    "cgl_gan_gather_buffers")
            self._gbufs = (self._wrap(s.value, n.value), self._wrap(r.value, max(self.n_workers, 1) * n.value))
        return self._gbufs

    def exchange_buffer(self):
        p, n = ctypes.c_void_p(), ctypes.c_int64()
        C.check(C.lib.cgl_gan_exchange_buffer(self._h, ctypes.byref(p), ctypes.byref(n)))
        return self._wrap(p.value, n.value)

    def g_output(self):
        """[2B, img] G output of the last round: rows < B = Xd, rows >= B = Xg."""
        p, n = ctypes.c_void_p(), ctypes.c_int64()
        C.check(C.lib.cgl_gan_tensor(self._h, 0, ctypes.byref(p), ctypes.byref(n)))
        return self._wrap(p.value, n.value).view(2 * self.B, -1)

    def internal(self, which):
        """Internal tensor by cgl_gan_tensor code (include/cglgan.h) as a flat float view."""
        p, n = ctypes.c_void_p(), ctypes.c_int64()
        C.check(C.lib.cgl_gan_tensor(self._h, which, ctypes.byref(p), ctypes.byref(n)), "cgl_gan_tensor")
        return self._wrap(p.value, n.value)

    def own_loss(self):
        p, n = ctypes.c_void_p(), ctypes.c_int64()
        C.check(C.lib.cgl_gan_tensor(self._h, 1, ctypes.byref(p), ctypes.byref(n)))
        return self._wrap(p.value, 1)

    def _wrap(self, addr, n):
        """View of a workspace region (the address lies inside self.workspace)."""
        base = self.workspace.data_ptr()
        off = addr - base
        if addr == 0 or off < 0 or off + 4 * n > self.workspace.numel():
            raise RuntimeError("address outside the context workspace")
        return self.workspace[off:off + 4 * n].view(torch.float32)

    def stats(self):
        s = C.GanStats()
        C.check(C.lib.cgl_gan_read_stats(self._h, ctypes.byref(s), _stream()), "cgl_gan_read_stats")
        return {"round": s.round, "d_loss": list(s.d_loss)[:self.epoch], "d_real": list(s.d_real)[:self.epoch],
                "d_fake": list(s.d_fake)[:self.epoch], "g_loss": s.g_loss, "alpha": s.alpha, "F": s.F,
                "lambda": s.lambda_, "bn_batches": s.bn_batches, "loss_scale": list(s.loss_scale),
                "last_skipped": list(s.last_skipped), "skipped": list(s.skipped)}

    def plan_info(self, phase=C.PHASE_ALL):
        nl, ng, fl = ctypes.c_int(), ctypes.c_int(), ctypes.c_double()
        C.check(C.lib.cgl_gan_plan_info(self._h, phase, ctypes.byref(nl), ctypes.byref(ng), ctypes.byref(fl)))
        return {"launches": nl.value, "gemm_launches": ng.value, "gemm_flops": fl.value}

    LAUNCH_KINDS = {0: "gemm", 1: "head", 2: "bn_bwd", 3: "adam", 4: "prologue", 5: "bn_apply", 6: "gemm_adam", 7: "gemm_prologue",
                    8: "alpha_combine"}

    def launches(self, phase=C.PHASE_ALL):
        """[(kind, flops, grid)] of the planned launches of a phase, in stream order."""
        n = C.lib.cgl_gan_launch_count(self._h, phase)
        out = []
        for i in range(n):
            k, f, g = ctypes.c_int(), ctypes.c_double(), ctypes.c_int()
            C.check(C.lib.cgl_gan_launch_info(self._h, phase, i, ctypes.byref(k), ctypes.byref(f), ctypes.byref(g)))
            out.append((self.LAUNCH_KINDS[k.value], f.value, g.value))
        return out

    def launch_one(self, idx, phase=C.PHASE_ALL):
        self._packed_current()
        C.check(C.lib.cgl_gan_launch_one(self._h, phase, idx, _stream()), "cgl_gan_launch_one")

    def profile_round(self, phase=C.PHASE_ALL):
        """One round (or phase) issued launch by launch with a start / stop event pair on every dispatch:
        [device microseconds of launch i] in plan order, measured in the round's own data state (each
        launch's inputs were just written by its producer, as in a replayed round).  Advances the training
        state like ``run``."""
        self._packed_current()
        n = C.lib.cgl_gan_launch_count(self._h, phase)
        buf = (ctypes.c_float * max(n, 1))()
        C.check(C.lib.cgl_gan_profile(self._h, phase, _stream(), buf, n), "cgl_gan_profile")
        return [float(buf[i]) for i in range(n)]

    def close(self):
        if getattr(self, "_h", None):
            C.lib.cgl_gan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
