"""One worker's CAPGAN round on the model/lsgan.py conv GAN, on its own MI355X.

The drop-in for the reference's Server.train + Worker.train pair (capgan.py:211-262 + :316-349)
with the conv Generator / Discriminator of model/lsgan.py:3-27, 73-99.  Every tensor operation is
a libcglgan_hip kernel (cglgan.conv_ops, stream-ordered, no host synchronisation inside a round);
the host only sequences launches.  The reference never trains these models, so the
adversarial objective is a knob: ``loss="mse"`` (LSGAN, D_loss = 0.5 (real + fake)) or ``"bce"``
(Sigmoid + BCELoss on the logit, D_loss = real + fake as in the BCE drivers).

Data layout (HBM, all NHWC fp32):
  G  (2B rows: the no-grad Xd call on z1, then the Xg call on z2 -- one launch chain, BatchNorm
     statistics per call):  z [2B,100] -> h [2B,8192] -> h0 [2B,8,8,128] -> y1/a1 [2B,16,16,128]
     -> y2/a2 [2B,32,32,64] -> x3[B:3B] (images, Tanh)
  x3 [3B,32,32,1]: rows [0,B) the sampled real batch, [B,2B) Xd, [2B,3B) Xg, so the D step reads
     [real; Xd] and the G-loss pass reads Xg without copies.
  D  (2B rows in the D step: the real call and the fake call, statistics and Dropout2d masks per
     call; B rows in the G-loss pass): q1..q4 (Conv -> LeakyReLU -> Dropout2d), r2..r4 (BN2d),
     flat [.,512] (NCHW flatten, model/lsgan.py:96), v [.,1]
Parameters: one flat buffer per model (+ grads, Adam m, v), 256-byte aligned tensors in
state-dict order, exposed as views under the reference's keys (``l1.0.weight``,
``conv_blocks.2.running_var``, ``model.14.bias``, ``adv_layer.weight`` ...).
"""
from __future__ import annotations

import math
import os
from collections import OrderedDict

import numpy as np
import torch

from . import _lib as C
from . import conv_ops as O

# (key, kind, shape) in construction (= state-dict) order, model/lsgan.py
LSGAN_G = [("l1.0", "linear", (128 * 8 * 8, 100)), ("conv_blocks.1", "conv", (128, 128)), ("conv_blocks.2", "bn", 128),
           ("conv_blocks.5", "conv", (64, 128)), ("conv_blocks.6", "bn", 64), ("conv_blocks.8", "conv", (1, 64))]
LSGAN_D = [("model.0", "conv", (16, 1)), ("model.3", "conv", (32, 16)), ("model.6", "bn", 32),
           ("model.7", "conv", (64, 32)), ("model.10", "bn", 64), ("model.11", "conv", (128, 64)),
           ("model.14", "bn", 128), ("adv_layer", "linear", (1, 128 * 2 * 2))]
D_CONVS = [("model.0", None, 1, 16, 32), ("model.3", "model.6", 16, 32, 16), ("model.7", "model.10", 32, 64, 8),
           ("model.11", "model.14", 64, 128, 4)]   # (conv, bn, cin, cout, input h = w)
DROP_P = 0.25
BN_EPS, BN_MOM, SLOPE = 0.8, 0.1, 0.2
_AL = 64   # floats: 256-byte tensor alignment


def tensor_shapes(spec):
    for key, kind, shp in spec:
        if kind == "linear":
            yield key + ".weight", tuple(shp), kind
            yield key + ".bias", (shp[0],), kind
        elif kind == "conv":
            yield key + ".weight", (shp[0], shp[1], 3, 3), kind
            yield key + ".bias", (shp[0],), kind
        else:
            yield key + ".weight", (shp,), kind
            yield key + ".bias", (shp,), kind


class FlatModel:
    """Flat parameter / grad / Adam-state buffers of one model with reference-keyed views."""

    def __init__(self, spec, device):
        self.spec = spec
        offs, off = [], 0
        for k, shp, _ in tensor_shapes(spec):
            n = math.prod(shp)
            offs.append((k, shp, off, n))
            off += (n + _AL - 1) // _AL * _AL
        f32 = dict(dtype=torch.float32, device=device)
        self.p, self.g = torch.zeros(off, **f32), torch.zeros(off, **f32)
        self.m, self.v = torch.zeros(off, **f32), torch.zeros(off, **f32)
        self.layout = offs
        self.params = OrderedDict((k, self.p[o:o + n].view(shp)) for k, shp, o, n in offs)
        self.grads = OrderedDict((k, self.g[o:o + n].view(shp)) for k, shp, o, n in offs)
        self._m = [self.m[o:o + n] for _, _, o, n in offs]
        self._v = [self.v[o:o + n] for _, _, o, n in offs]
        self.running = OrderedDict()
        self.batches = OrderedDict()
        for key, kind, shp in spec:
            if kind == "bn":
                self.running[key + ".running_mean"] = torch.zeros(shp, **f32)
                self.running[key + ".running_var"] = torch.ones(shp, **f32)
                self.batches[key] = 0
        self.step = 0

    def adam(self, lr, betas, eps, step_dev=None):
        """step_dev: device int32 holding the completed steps (the graph-replayable round reads the
        step there); the host count advances either way."""
        self.step += 1
        ps = [self.params[k].view(-1) for k, _, _, _ in self.layout]
        gs = [self.grads[k].view(-1) for k, _, _, _ in self.layout]
        O.adam_multi(ps, gs, self._m, self._v, self.step, lr, betas, eps, step_dev=step_dev)

    def state_dict(self):
        sd = OrderedDict()
        for key, kind, _ in self.spec:
            sd[key + ".weight"] = self.params[key + ".weight"].detach().clone()
            sd[key + ".bias"] = self.params[key + ".bias"].detach().clone()
            if kind == "bn":
                sd[key + ".running_mean"] = self.running[key + ".running_mean"].clone()
                sd[key + ".running_var"] = self.running[key + ".running_var"].clone()
                sd[key + ".num_batches_tracked"] = torch.tensor(self.batches[key], dtype=torch.long)
        return sd

    @torch.no_grad()
    def load_state_dict(self, sd):
        for k, v in self.params.items():
            v.copy_(sd[k].reshape(v.shape))
        for k, v in self.running.items():
            if k in sd:
                v.copy_(sd[k])
        for key in self.batches:
            if key + ".num_batches_tracked" in sd:
                self.batches[key] = int(sd[key + ".num_batches_tracked"])
        self.m.zero_()
        self.v.zero_()
        self.step = 0


@torch.no_grad()
def default_init(fm: FlatModel, generator=None):
    """nn.Linear / nn.Conv2d reset_parameters (kaiming_uniform_(a=sqrt(5)); bias U(+-1/sqrt(fan_in))) and
    BatchNorm2d (1, 0), drawn from the torch CPU RNG in construction order: torch.manual_seed(s) then
    this equals torch.manual_seed(s); Generator(ims) / Discriminator(ims) of model/lsgan.py."""
    for key, kind, shp in fm.spec:
        w, b = fm.params[key + ".weight"], fm.params[key + ".bias"]
        if kind == "bn":
            w.fill_(1.0)
            b.fill_(0.0)
            continue
        wc = torch.empty(w.shape)
        bc = torch.empty(b.shape)
        torch.nn.init.kaiming_uniform_(wc, a=math.sqrt(5), generator=generator)
        bound = 1.0 / math.sqrt(wc[0].numel())
        torch.nn.init.uniform_(bc, -bound, bound, generator=generator)
        w.copy_(wc)
        b.copy_(bc)


class ConvGanStep:
    """Fused CAPGAN worker round of the model/lsgan.py GAN (see module docstring)."""

    def __init__(self, batch, loss="mse", data=None, seed=20211212, n_workers=1, rank=0, weighting="capgan",
                 lr=2e-4, betas=(0.5, 0.999), adam_eps=1e-8, gen_z=True, beta=None, device="cuda", graph=False):
        if loss not in ("mse", "bce"):
            raise ValueError("loss must be 'mse' (LSGAN) or 'bce' (Sigmoid + BCELoss)")
        if batch < 2:
            raise ValueError("BatchNorm in train mode needs batch >= 2")
        dev = torch.device(device)
        self.device, self.B, self.loss = dev, batch, loss
        self.lr, self.betas, self.eps = lr, betas, adam_eps
        self.seed, self.gen_z = seed, gen_z
        self.n_workers, self.rank, self.weighting = n_workers, rank, weighting
        self.G, self.D = FlatModel(LSGAN_G, dev), FlatModel(LSGAN_D, dev)
        B, B2 = batch, 2 * batch
        e = lambda *s: torch.zeros(*s, dtype=torch.float32, device=dev)
        self.z = e(B2, 100)
        self.h, self.h0 = e(B2, 8192), e(B2, 8, 8, 128)
        self.y1, self.a1 = e(B2, 16, 16, 128), e(B2, 16, 16, 128)
        self.y2, self.a2 = e(B2, 32, 32, 64), e(B2, 32, 32, 64)
        self.x3 = e(3 * B, 32, 32, 1)
        self.g_save = {k: (e(2, c), e(2, c)) for k, c in (("conv_blocks.2", 128), ("conv_blocks.6", 64))}
        # D activations (2B rows: D step; first B rows reused by the G-loss pass)
        self.q = [e(B2, hw // 2, hw // 2, co) for _, _, _, co, hw in D_CONVS]
        self.r = [None] + [e(B2, hw // 2, hw // 2, co) for _, _, _, co, hw in D_CONVS[1:]]
        self.flat, self.v = e(B2, 512), e(B2, 1)
        self.d_save = {bn: (e(2, co), e(2, co)) for _, bn, _, co, _ in D_CONVS if bn}
        self.mask_d = [e(B2, co) for _, _, _, co, _ in D_CONVS]    # D step masks (real rows, then fake rows)
        self.mask_g = [e(B, co) for _, _, _, co, _ in D_CONVS]     # G-loss pass masks
        # gradients
        self.dv = e(B2, 1)
        self.dr = [None] + [e(B2, hw // 2, hw // 2, co) for _, _, _, co, hw in D_CONVS[1:]]
        self.dc = [e(B2, hw // 2, hw // 2, co) for _, _, _, co, hw in D_CONVS]
        self.dq1 = e(B2, 16, 16, 16)
        self.dimg, self.dc3g = e(B, 32, 32, 1), e(B, 32, 32, 1)
        self.da2, self.dy2 = e(B, 32, 32, 64), e(B, 32, 32, 64)
        self.da1, self.dy1 = e(B, 16, 16, 128), e(B, 16, 16, 128)
        self.dh0, self.dh = e(B, 8, 8, 128), e(B, 8192)
        self.lbuf = e(8)                       # d_real, d_fake, g_loss
        self.losses_all = e(max(n_workers, 1))
        self.lam = 0.0
        self.beta = None
        self.set_beta(beta)
        self.round = 0
        # graph=True: every per-round value comes from the device counter block `dstate` (round, G
        # Adam steps, D Adam steps) -- z stream, Dropout2d counters, Adam bias corrections, and the
        # real batch through the device sampler (cgl_sample_rows_dev) -- and run() replays one
        # captured round as a hipGraph (N = 1; phases stay eager for the multi-worker exchange)
        self.graph = bool(graph)
        self.dstate = torch.zeros(5, dtype=torch.int32, device=dev)
        # dstate[4]: the G steps completed before this round's G Adam (written by the G backward's deferred launch
        # when it also advances the counters: CGL_CONV_CNTFOLD, one cgl_counters_add launch fewer per round)
        # dstate[3]: real images of this round's D-step real call (DataLoader's short final batch of a pass,
        # capgan.py:282,326-331: a shard of n rows gives ceil(n / B) batches per pass, the last n mod B rows);
        # the D-step kernels leave the padding images of a short call out (nvalid)
        self.nv = self.dstate[3:4]
        self.nv.fill_(batch)
        self._dstate_host = (0, 0, 0)         # host mirror of dstate after the last issued round
        self._cuda_graph = None
        self._kgraphs = {}             # rounds -> graph of that many whole rounds (run_rounds)
        self._phase_graphs = None      # (phase A, phase B) graphs of the split round (N > 1)
        self._split_graph = False
        self._graph_delta = None
        # packed MFMA weight operands of every layer (cglgan.conv_ops.PackSet): G and D are packed
        # together at the start of a round (the exchanges between rounds may rewrite either), D again
        # after its Adam step -- two pack launches per round instead of one per conv call
        PG, PD = self.G.params, self.D.params
        pk = O.PackSet()
        pk.add("G", "c1f", PG["conv_blocks.1.weight"], 8, 8, 128, 128, 1, 1)
        pk.add("G", "c1b", PG["conv_blocks.1.weight"], 8, 8, 128, 128, 1, 1, dir=1)
        pk.add("G", "c5f", PG["conv_blocks.5.weight"], 16, 16, 128, 64, 1, 1)
        pk.add("G", "c5b", PG["conv_blocks.5.weight"], 16, 16, 128, 64, 1, 1, dir=1)
        pk.add("G", "c8f", PG["conv_blocks.8.weight"], 32, 32, 64, 1, 1, 0)
        # the Linear(100, 8192) works on the NHWC activation directly (CGL_CONV_L1NHWC): forward output column
        # n = hw * 128 + c gathers W row c * 64 + hw, and its bias is packed in that order with the G operands
        # (the 1x1 input-gradient pack of a [128][64] "weight" is its transpose); the weight gradient reads the
        # NHWC gradient and stores its rows in the reference's order -- no transpose launch either way
        self.l1nhwc = os.environ.get("CGL_CONV_L1NHWC", "1") != "0"
        if self.l1nhwc:
            pk.add("G", "l1b", PG["l1.0.bias"], 1, 1, 64, 128, 1, 0, ks=1, dir=1)
        for ck, _, ci, co, hw in D_CONVS:
            pk.add("D", ck + "f", PD[ck + ".weight"], hw, hw, ci, co, 2, 0)
            pk.add("D", ck + "b", PD[ck + ".weight"], hw, hw, ci, co, 2, 0, dir=1)
        self.pk = pk.finalize(dev)
        # G's nn.Linear(100, 8192) (model/lsgan.py:8) on the fused-MLP GEMM kernel, prepared once:
        # forward on [z1; z2] and its weight + bias gradient on the z2 rows
        GG = self.G.grads
        if self.l1nhwc:
            n = torch.arange(8192, dtype=torch.int32, device=dev)
            self.l1_rows = ((n % 128) * 64 + n // 128).to(torch.int32).contiguous()
            self.l1_fwd = O.PreparedLinear(0, self.z, PG["l1.0.weight"], self.pk["l1b"], self.h0, None, B2, 8192, 100,
                                           b_rows=self.l1_rows)
        else:
            self.l1_fwd = O.PreparedLinear(0, self.z, PG["l1.0.weight"], PG["l1.0.bias"], self.h, None, B2, 8192, 100)
        if self.l1nhwc:   # its weight + bias gradient read the NHWC gradient dh0 (output rows permuted at the store)
            self.l1_wgrad = O.PreparedLinear(2, self.dh0, self.z[B:], None, GG["l1.0.weight"], GG["l1.0.bias"], B, 8192,
                                             100, nhwc=(128, 64))
        else:
            self.l1_wgrad = O.PreparedLinear(2, self.dh, self.z[B:], None, GG["l1.0.weight"], GG["l1.0.bias"], B, 8192,
                                             100)
        # BatchNorm2d statistics written by the producing conv's epilogue (cgl_conv3x3_fwd_packed_stats):
        # one float64 partial buffer per BatchNorm, sized for its largest call (the D step's 2B rows)
        sc = lambda n, h, ci, co, st, up, grp: O.stat_chunks(n, h, h, ci, co, st, up, grp)
        self.st_geo = {"conv_blocks.2": (B2, 8, 128, 128, 1, 1, 2), "conv_blocks.6": (B2, 16, 128, 64, 1, 1, 2)}
        for ck, bk, ci, co, hw in D_CONVS:
            if bk:
                self.st_geo[bk] = (B2, hw, ci, co, 2, 0, 2)
        self.st_part, self.st_scratch = {}, {}
        for k, geo in self.st_geo.items():
            n = sc(*geo)
            if n > 0:
                self.st_part[k] = torch.zeros(n * geo[3] * 2, dtype=torch.float64, device=dev)
                self.st_scratch[k] = O.bn2d_stats_scratch(geo[3], geo[6], dev)
        # G BatchNorm2d + LeakyReLU folded into the next conv's operand load (model/lsgan.py:15-22): the finalize
        # keeps scale / shift per (forward call, channel) [2][2][C].  CGL_CONV_BNFOLD = bit mask (1: conv_blocks.2
        # into the up-convolution conv_blocks.5, 2: conv_blocks.6 into conv_blocks.8), default 2: the up-convolution
        # reads each input 16 times (4 output parities x 4 taps), so its fold re-applies the BatchNorm 16 times per
        # element and measured slower than the separate pass (profiles/r03_conv_bnfold_ab.txt)
        # CGL_CONV_ELIDE (default 1): with a layer folded, its activation is not stored at all -- the G backward
        # applies the BatchNorm in the weight gradient's operand loads (cgl_conv3x3_bwd_weight_bnin) and takes
        # LeakyReLU' from the kept scale / shift.  Measured (profiles/r04_conv_elide_ab.txt): a2 (fold bit 2)
        # -28 us per round; a1 too (bit 1) another -6 us once the BatchNorm-in-load paths keep the activation
        # flag and slope in registers, so with the elision the default mask is 3 (2 without it)
        self.elide_on = os.environ.get("CGL_CONV_ELIDE", "1") != "0"
        fold = int(os.environ.get("CGL_CONV_BNFOLD", "3" if self.elide_on else "2"))
        self.bn_fold = fold & 3 if all(k in self.st_part for k in ("conv_blocks.2", "conv_blocks.6")) else 0
        self.coef = {k: torch.zeros(4 * c, dtype=torch.float32, device=dev)
                     for k, c in (("conv_blocks.2", 128), ("conv_blocks.6", 64))}
        # the G backward takes LeakyReLU'(a) of these BatchNorms from the sign of the kept scale / shift applied
        # to y (cgl_bn2d_bwd post_coef) instead of reading a: bitwise the same mask, one tensor fewer read in the
        # channel reduction and in the backward apply (CGL_CONV_POSTCOEF=0 reads a)
        self.coef_kept = set()
        # D's inner BatchNorms folded into the next conv in the G-loss pass (_d_forward); [2][groups][C] scale / shift
        self.d_fold = os.environ.get("CGL_CONV_DFOLD", "1") != "0"
        self.batch_on = os.environ.get("CGL_CONV_BATCH", "1") != "0"   # batched round start (_phase_a)
        # ... and in the D step too (CGL_CONV_DFOLD_STEP=1): correct and bitwise, but the wave-unit weight gradient's
        # per-value BatchNorm costs +41 us against the two apply passes it saves (profiles/r04_conv_elide_ab.txt)
        self.d_fold_step = os.environ.get("CGL_CONV_DFOLD_STEP", "0") == "1"
        self._d_folded = set()   # D-step BatchNorms folded this round (their weight gradients apply them)
        self.dcoef = {bk: torch.zeros(4 * co, dtype=torch.float32, device=dev) for _, bk, _, co, _ in D_CONVS if bk}
        self.post_coef_on = os.environ.get("CGL_CONV_POSTCOEF", "1") != "0"
        # backward statistics: the same buffers (the forward's partials are consumed by then), written
        # by the input-gradient conv that produces the BatchNorm's output gradient
        self.bst_ok = {}
        bgeo = {"conv_blocks.2": (B, 16, 128, 64, 1, 1, 1)}     # conv_blocks.5 input gradient -> da1
        for k in range(2, 4):
            ck, _, ci, co, hw = D_CONVS[k]
            bgeo[D_CONVS[k - 1][1]] = (B2, hw, ci, co, 2, 0, 2)   # conv k input gradient -> dr[k - 1]
        for key, (n, h, ci, co, st, up, grp) in bgeo.items():
            nb = O.stat_chunks(n, h, h, ci, co, st, up, grp, bwd=True)
            self.bst_ok[key] = key in self.st_part and 0 < nb * ci * 2 <= self.st_part[key].numel()
        # conv_blocks.6's backward partials from the Conv2d(64, 1) input gradient itself (cgl_conv3x3_bwd_data_stats,
        # 128-row chunks: bitwise the channel reduction it saves; CGL_CONV_N1STATS=0 keeps that launch).  Only where
        # that reduction itself uses 128-row chunks (the library's chan_chunk halves them below CGL_CHAN_MINCH = 64
        # chunks per call, i.e. B < 8), so both paths stay bitwise equal at every batch
        minch = int(os.environ.get("CGL_CHAN_MINCH", "64"))
        self.n1_stats = (os.environ.get("CGL_CONV_N1STATS", "1") != "0" and "conv_blocks.6" in self.st_part and
                         B * 1024 % 128 == 0 and B * 1024 // 128 >= minch and
                         B * 1024 // 128 * 64 * 2 <= self.st_part["conv_blocks.6"].numel())
        # D's Conv2d(1, 16) weight gradient applies its block's LeakyReLU + Dropout2d backward in its loads in the D
        # step (cgl_conv3x3_bwd_weight_actdrop; bitwise, one launch fewer; CGL_CONV_C1FUSE=0 keeps act_drop_bwd)
        self.c1_fuse = os.environ.get("CGL_CONV_C1FUSE", "1") != "0"
        # the D head (adv_layer forward, the loss head(s), adv_layer's input gradient) as ONE launch per pass
        # (cgl_dense1_head_nhwc, bitwise the separate launches; CGL_CONV_HEADFUSE=0 keeps them).  Each pass has its
        # own scratch: a monotonic ticket counted modulo that launch's grid + the per-row loss terms
        self.head_fuse = os.environ.get("CGL_CONV_HEADFUSE", "1") != "0"
        # ... and with it, D's last BatchNorm (model.14) applied in the head's loads (its finalize keeps the scale /
        # shift only: one cgl_eltwise fewer per pass; bitwise, CGL_CONV_HEADBN=0 applies it)
        self.head_bn = self.head_fuse and os.environ.get("CGL_CONV_HEADBN", "1") != "0"
        self._head_coef = None
        self.hscr_d, self.hscr_g = torch.zeros(B2 + 16, device=dev), torch.zeros(B + 16, device=dev)
        # the split reductions of a backward pass's weight gradients (and Conv2d(1, 16)'s finish) as ONE launch at the
        # end of the pass (cgl_conv_wgrad_defer; bitwise the separate launches; CGL_CONV_WDEFER=0 launches each with
        # its MFMA kernel): every deferred weight gradient writes its partials into a workspace of its own
        # the G BatchNorm backward applies (conv_blocks.6 / .2, from producer statistics) also write their output's
        # column sums per 256-row chunk: conv_blocks.5 / .1's bias gradients without their own pass over dy2 / dy1
        # (cgl_bn2d_bwd_stats colsum_part + cgl_colsum_finalize; bitwise; CGL_CONV_BNBCOL=0: the weight gradient's)
        # (only where the weight gradient itself sums columns of dY: cgl_conv3x3_bias_by_colsum)
        self.bnb_col = os.environ.get("CGL_CONV_BNBCOL", "1") != "0"
        self.bcs = {}
        for k, hw, c, geo in (("conv_blocks.6", 1024, 64, (B, 16, 16, 128, 64, 1, 1)),
                              ("conv_blocks.2", 256, 128, (B, 8, 8, 128, 128, 1, 1))):
            if self.bnb_col and C.lib.cgl_conv3x3_bias_by_colsum(*geo) == 1:
                self.bcs[k] = torch.zeros(B * hw // 256 * c * 2, dtype=torch.float64, device=dev)
        self.wdefer = os.environ.get("CGL_CONV_WDEFER", "1") != "0"
        self.cnt_fold = os.environ.get("CGL_CONV_CNTFOLD", "1") != "0"
        self.wws = {}
        if self.wdefer:
            geoms = {ck: (B2, hw, hw, ci, co, 2, 0) for ck, _, ci, co, hw in D_CONVS}
            geoms.update({"conv_blocks.8": (B, 32, 32, 64, 1, 1, 0), "conv_blocks.5": (B, 16, 16, 128, 64, 1, 1),
                          "conv_blocks.1": (B, 8, 8, 128, 128, 1, 1)})
            for k, geo in geoms.items():
                self.wws[k] = torch.empty(O.conv_ws_bytes(*geo), dtype=torch.uint8, device=dev)
        self.bpart = (torch.zeros(2 * (B * 1024 // 256), dtype=torch.float64, device=dev)
                      if os.environ.get("CGL_CONV_BIASFUSE", "1") != "0" and B * 1024 % 256 == 0 and B <= 2048 else None)
        # sampler over a device-resident real shard [n, 1024] (DataLoader(shuffle=True), capgan.py:282)
        self.data = data
        self.short = data is not None and data.shape[0] % batch != 0    # some batch of a pass is short
        self._short_call = False          # this round's real call may be short (nvalid passed to the D step)
        self._perm, self._pos = None, 0
        self._gen = torch.Generator().manual_seed(seed + 1 + rank)
        if data is not None:
            if data.dim() != 2 or data.shape[1] != 1024 or data.shape[0] < 1:
                raise ValueError("data must be a [n >= 1, 1024] tensor of 32x32 images")
            if not data.is_cuda or data.dtype != torch.float32:
                raise ValueError("data must be float32 on the GPU")

    # ------------------------------------------------------------------ state
    def set_beta(self, beta=None):
        """Data-size weights of the CAPGAN alpha (capgan.py:149-153: beta_c = len(shard_c) / sum; see
        cglgan.data.beta_weights); None = equal shards (1 / N each)."""
        b = [1.0 / self.n_workers] * self.n_workers if beta is None else [float(x) for x in beta]
        if len(b) != self.n_workers:
            raise ValueError(f"beta needs one weight per worker ({self.n_workers})")
        self.beta = b

    def init_default(self, seed_g=20211212, seed_d=None):
        """capgan.py:28,156,309: torch.manual_seed(seed) then G (and D) constructed."""
        torch.manual_seed(seed_g)
        default_init(self.G)
        if seed_d is not None:
            torch.manual_seed(seed_d)
        default_init(self.D)

    # ------------------------------------------------------------------ resume
    def resume_state(self):
        """Everything the next round reads: G / D parameters and Adam moments, BatchNorm running
        statistics and batch counts, Adam steps, the round counter (z stream, Dropout2d counters),
        lambda and the real-batch sampler (permutation, position, its generator) as CPU tensors."""
        torch.cuda.current_stream().synchronize()
        out = OrderedDict()
        for tag, fm in (("G", self.G), ("D", self.D)):
            for k in ("p", "m", "v"):
                out[f"{tag}.{k}"] = getattr(fm, k).detach().cpu().clone()
            for k, v in fm.running.items():
                out[f"{tag}.running.{k}"] = v.detach().cpu().clone()
            out[f"{tag}.batches"] = torch.tensor([fm.batches[k] for k in fm.batches], dtype=torch.long)
            out[f"{tag}.step"] = torch.tensor(fm.step, dtype=torch.long)
        out["round"] = torch.tensor(self.round, dtype=torch.long)
        out["lam"] = torch.tensor(self.lam, dtype=torch.float64)
        out["sampler.pos"] = torch.tensor(self._pos, dtype=torch.long)
        out["sampler.perm"] = (self._perm.cpu().clone() if self._perm is not None else torch.zeros(0, dtype=torch.int32))
        out["sampler.gen"] = self._gen.get_state()
        return out

    @torch.no_grad()
    def load_resume_state(self, sd):
        for tag, fm in (("G", self.G), ("D", self.D)):
            for k in ("p", "m", "v"):
                getattr(fm, k).copy_(sd[f"{tag}.{k}"])
            for k, v in fm.running.items():
                v.copy_(sd[f"{tag}.running.{k}"])
            for k, b in zip(list(fm.batches), sd[f"{tag}.batches"].tolist()):
                fm.batches[k] = int(b)
            fm.step = int(sd[f"{tag}.step"])
        self.round = int(sd["round"])
        self.lam = float(sd["lam"])
        self._pos = int(sd["sampler.pos"])
        perm = sd["sampler.perm"]
        self._perm = perm.to(self.device) if perm.numel() else None
        self._gen.set_state(sd["sampler.gen"])
        self._dstate_host = None            # rewritten from the host state by the next round
        torch.cuda.current_stream().synchronize()

    # ------------------------------------------------------------------ pieces
    def _sample_real(self):
        """DataLoader(shuffle=True) over the shard (capgan.py:282,326-331): a fresh permutation per pass, cut
        into batches of B, the pass's last batch short (n mod B rows); its padding rows repeat a real row."""
        B = self.B
        n = self.data.shape[0]
        if self._perm is None or self._pos >= n:
            self._perm = torch.randperm(n, generator=self._gen).to(torch.int32).to(self.device, non_blocking=True)
            self._pos = 0
        take = min(B, n - self._pos)
        idx = self._perm[self._pos:self._pos + take]
        if take < B:
            idx = torch.cat([idx, idx[:1].expand(B - take)])
        O.gather_rows(self.data, idx, 0, B, 1024, self.x3)
        if self.short:
            self.nv.fill_(take)
        self._pos += take

    def _g_forward(self):
        P, B2 = self.G.params, 2 * self.B
        self.l1_fwd()
        if not self.l1nhwc:
            O.nchw_to_nhwc(self.h, self.h0, B2, 128, 64)      # out.view(B, 128, 8, 8), model/lsgan.py:25
        O.conv3x3_fwd(self.h0, P["conv_blocks.1.weight"], P["conv_blocks.1.bias"], self.y1, B2, 8, 8, 128, 128, 1, 1,
                      wp=self.pk["c1f"], stats=self._stats("conv_blocks.2", 2))
        # BatchNorm2d + LeakyReLU of y1 (bit 0) / y2 (bit 1) folded into the next conv's operand load (the finalize
        # keeps the scale / shift); a folded layer's activation is written for the Xg half only (images B .. 2B),
        # which the G backward reads
        f1, f2 = bool(self.bn_fold & 1), bool(self.bn_fold & 2)
        bi = lambda k: (self.coef[k], 2, O.ACT_LEAKY, SLOPE)
        self._g_bn("conv_blocks.2", self.y1, self.a1, 256, 128, fold=f1)
        O.conv3x3_fwd(self.y1 if f1 else self.a1, P["conv_blocks.5.weight"], P["conv_blocks.5.bias"], self.y2, B2, 16,
                      16, 128, 64, 1, 1, wp=self.pk["c5f"], stats=self._stats("conv_blocks.6", 2),
                      bn_in=bi("conv_blocks.2") if f1 else None)
        self._g_bn("conv_blocks.6", self.y2, self.a2, 1024, 64, fold=f2)
        O.conv3x3_fwd(self.y2 if f2 else self.a2, P["conv_blocks.8.weight"], P["conv_blocks.8.bias"], self.x3[self.B:],
                      B2, 32, 32, 64, 1, 1, 0, act=O.ACT_TANH, wp=self.pk["c8f"],
                      bn_in=bi("conv_blocks.6") if f2 else None)

    def g_act_xd(self, name):
        """The Xd half (images 0 .. B) of a1 / a2 (see g_act)."""
        return self.g_act(name)[:self.B]

    def g_act(self, name):
        """a1 / a2 over both calls (images 0 .. 2B): the stored tensor where the forward wrote it; with the
        BatchNorm fold (the consumer conv applied it in its loads) the Xd half, and with the elision
        (CGL_CONV_ELIDE) both halves, recomputed here from y and the kept scale / shift in double -- for
        inspection (signs, values), not used by the round."""
        y, a, key, bit = ((self.y1, self.a1, "conv_blocks.2", 1) if name == "a1" else
                          (self.y2, self.a2, "conv_blocks.6", 2))
        if not (self.bn_fold & bit):
            return a
        c, B = y.shape[-1], self.B

        def rec(g, rows):
            sc, sh = self.coef[key][g * c:(g + 1) * c].double(), self.coef[key][(2 + g) * c:(3 + g) * c].double()
            v = rows.double() * sc + sh
            return torch.where(v > 0, v, v * SLOPE).float()
        xg = rec(1, y[B:]) if self._elided(key) else a[B:]
        return torch.cat([rec(0, y[:B]), xg])

    def _stats(self, key, groups):
        part = self.st_part.get(key)
        return (part, groups) if part is not None else None

    def _bn_fwd(self, key, fm, x, y, n, hw, c, groups, act, fold=False, nvalid=None, coef_only=False):
        """BatchNorm2d (train) from the partials the producing conv wrote, else with its own pass.
        ``fold``: keep the scale / shift in self.coef[key] and apply to the last group (Xg) only."""
        P, R = fm.params, fm.running
        sm, si = (self.g_save if fm is self.G else self.d_save)[key]
        kw = dict(groups=groups, eps=BN_EPS, momentum=BN_MOM, running_mean=R[key + ".running_mean"],
                  running_var=R[key + ".running_var"], act=act, slope=SLOPE, save_mean=sm, save_invstd=si,
                  nvalid=nvalid)
        if coef_only:     # the consumer conv applies it (bn_in): keep scale / shift, write no activation
            kw.update(coef=(self.coef if key in self.coef else self.dcoef)[key], apply_from=n)
        elif fold:
            kw.update(coef=self.coef[key], apply_from=n - n // groups)
        elif key in self.coef and key in self.st_part:
            kw.update(coef=self.coef[key], apply_from=0)     # applied to every call, scale / shift kept
        if key in self.coef and key in self.st_part:
            self.coef_kept.add(key)
        if key in self.st_part:
            O.bn2d_fwd_stats(self.st_part[key], x, n, hw, c, P[key + ".weight"], P[key + ".bias"], y,
                             scratch=self.st_scratch[key], **kw)
        else:
            O.bn2d_fwd(x, n, hw, c, P[key + ".weight"], P[key + ".bias"], y, train=True, **kw)
        fm.batches[key] += groups

    def _post_coef(self, key):
        """(coef, group 1 = Xg, 2 calls) for cgl_bn2d_bwd's post_coef when this round's forward kept them."""
        return (self.coef[key], 1, 2) if (self.post_coef_on and key in self.coef_kept) else None

    def _g_bn(self, key, x, y, hw, c, fold=False):
        self._bn_fwd(key, self.G, x, y, 2 * self.B, hw, c, 2, O.ACT_LEAKY, fold=fold,
                     coef_only=fold and self._elided(key))

    def _elided(self, key):
        """The G activation after BatchNorm ``key`` is never stored (folded forward + BNIN weight gradient +
        LeakyReLU' from the kept scale / shift); needs the post-coefficient path on."""
        bit = 1 if key == "conv_blocks.2" else 2
        return bool(self.elide_on and self.post_coef_on and (self.bn_fold & bit))

    def _masks(self):
        """Every Dropout2d mask of the round in one launch: the D step's (call 0, 2B images) and the
        G-loss pass's (call 1, B images); counter (round * 2 + call) * 4 + layer."""
        B, cs = self.B, [co for _, _, _, co, _ in D_CONVS]
        if self.graph:      # counter = (round * 2 + call) * 4 + k with the round read on the device
            O.dropout2d_masks_dev(self.mask_d + self.mask_g, [2 * B] * 4 + [B] * 4, cs + cs, DROP_P,
                                  self.seed * 7919 + self.rank, [call * 4 + k for call in (0, 1) for k in range(4)],
                                  self.dstate[0:1], 8)
            return
        O.dropout2d_masks(self.mask_d + self.mask_g, [2 * B] * 4 + [B] * 4, cs + cs, DROP_P,
                          self.seed * 7919 + self.rank,
                          [(self.round * 2 + call) * 4 + k for call in (0, 1) for k in range(4)])

    def _d_forward(self, x, n, groups, masks, nvalid=None):
        """``nvalid``: the first call (the real images) is a short batch of *nvalid images.
        Each inner BatchNorm2d is folded into the next conv's operand load (bn_in) and writes no activation:
        in the G-loss pass nothing else reads it; in the D step (opt-in, d_fold_step) the next conv's weight
        gradient applies it in its operand loads too (cgl_conv3x3_bwd_weight_bnin) -- two cgl_eltwise passes fewer
        per pass; CGL_CONV_DFOLD=0 applies them."""
        P, R = self.D.params, self.D.running
        self._head_coef = None
        fold_pass = self.d_fold and ((masks is self.mask_g and groups == 1) or
                                     (masks is self.mask_d and self.d_fold_step))
        if masks is self.mask_d:
            self._d_folded = set()
        inp, bn_in = x, None
        for k, (ck, bk, ci, co, hw) in enumerate(D_CONVS):
            st = self._stats(bk, groups) if bk else None
            O.conv3x3_fwd(inp, P[ck + ".weight"], P[ck + ".bias"], self.q[k], n, hw, hw, ci, co, 2, 0, act=O.ACT_LEAKY,
                          slope=SLOPE, drop=masks[k], wp=self.pk[ck + "f"], stats=st,
                          nvalid=nvalid if st is not None else None, bn_in=bn_in)
            inp, bn_in = self.q[k], None
            if bk:
                last = k + 1 == len(D_CONVS)
                hfold = last and self.head_bn and bk in self.st_part     # the head applies it
                fold = (fold_pass and not last and bk in self.st_part) or hfold
                self._bn_fwd(bk, self.D, self.q[k], self.r[k], n, (hw // 2) ** 2, co, groups, O.ACT_NONE, nvalid=nvalid,
                             coef_only=fold)
                if hfold:
                    self._head_coef = (self.dcoef[bk], groups)
                elif fold:
                    bn_in = (self.dcoef[bk], groups, O.ACT_NONE, SLOPE)
                    if masks is self.mask_d:
                        self._d_folded.add(bk)
                else:
                    inp = self.r[k]
        # out.view(B, -1) -> adv_layer (model/lsgan.py:96-97) from the NHWC map; the D step's call keeps the
        # NCHW view for adv_layer's weight gradient, the G-loss pass (no D weight gradient) does not
        if not self.head_fuse:      # (fused: the head launch of _head computes it)
            O.dense1_fwd_nhwc(self.r[3], P["adv_layer.weight"], P["adv_layer.bias"], self.v, n, 128, 4,
                              flat=self.flat if masks is self.mask_d else None)

    def _head(self, n, calls, scratch, flat):
        """adv_layer forward + the loss head(s) + adv_layer's input gradient (dr[3]) as one launch."""
        P = self.D.params
        hc = self._head_coef if self.head_bn else None
        O.dense1_head_nhwc(self.q[3] if hc else self.r[3], P["adv_layer.weight"], P["adv_layer.bias"], self.v, self.dv,
                           self.dr[3], n, 128, 4, self.loss, calls, scratch, flat=flat, bn_in=hc)

    def _d_backward(self, x, n, groups, masks, wgrad, dx, nvalid=None):
        with O.wgrad_defer(wgrad and self.wdefer):
            self._d_backward_ops(x, n, groups, masks, wgrad, dx, nvalid)

    def _d_backward_ops(self, x, n, groups, masks, wgrad, dx, nvalid=None):
        P, G = self.D.params, self.D.grads
        wws = self.wws if wgrad else {}
        bst = set()     # BatchNorms whose backward partials the previous input-gradient conv wrote
        if not self.head_fuse:      # (fused: the head launch wrote dr[3])
            O.dense1_bwd_data_nhwc(self.dv, P["adv_layer.weight"], self.dr[3], n, 128, 4)
        if wgrad:
            O.dense_bwd_weight(self.dv, self.flat, G["adv_layer.weight"], G["adv_layer.bias"], n, 512, 1)
        c1f = False
        for k in (3, 2, 1, 0):
            ck, bk, ci, co, hw = D_CONVS[k]
            ho = hw // 2
            if bk:
                sm, si = self.d_save[bk]
                kw = dict(groups=groups, post_out=self.q[k], drop=masks[k], dgamma=G[bk + ".weight"] if wgrad else None,
                          dbeta=G[bk + ".bias"] if wgrad else None, slope=SLOPE, nvalid=nvalid)
                if bk in bst:
                    O.bn2d_bwd_stats(self.st_part[bk], self.dr[k], self.q[k], n, ho * ho, co, sm, si, P[bk + ".weight"],
                                     self.dc[k], **kw)
                else:
                    O.bn2d_bwd(self.dr[k], self.q[k], n, ho * ho, co, sm, si, P[bk + ".weight"], self.dc[k], **kw)
            elif not (c1f := wgrad and dx is None and self.c1_fuse):
                O.act_drop_bwd(self.dq1, self.q[0], masks[0], n, ho * ho, co, self.dc[0], slope=SLOPE)
            inp = x if k == 0 else (self.q[0] if k == 1 else self.r[k - 1])
            pfold = k > 1 and D_CONVS[k - 1][1] in self._d_folded
            if k == 0 and not bk and c1f:   # dc[0] only feeds this weight gradient: its act / drop backward in the loads
                O.conv3x3_bwd_weight(self.dq1, inp, G[ck + ".weight"], G[ck + ".bias"], n, hw, hw, ci, co, 2, 0,
                                     act_drop=(self.q[0], masks[0], SLOPE), ws=wws.get(ck))
            elif wgrad and pfold:     # r[k - 1] = BN(q[k - 1]) applied in the operand loads (both calls of the step)
                O.conv3x3_bwd_weight(self.dc[k], self.q[k - 1], G[ck + ".weight"], G[ck + ".bias"], n, hw, hw, ci, co,
                                     2, 0, bn_in=(self.dcoef[D_CONVS[k - 1][1]], -1, groups, O.ACT_NONE, SLOPE),
                                     ws=wws.get(ck))
            elif wgrad:
                O.conv3x3_bwd_weight(self.dc[k], inp, G[ck + ".weight"], G[ck + ".bias"], n, hw, hw, ci, co, 2, 0,
                                     ws=wws.get(ck))
            if k > 0:
                pbk = D_CONVS[k - 1][1]
                st = None
                if k > 1 and self.bst_ok.get(pbk):
                    st = (self.st_part[pbk], groups, self.q[k - 1], None, self.d_save[pbk][0], SLOPE)
                    bst.add(pbk)
                O.conv3x3_bwd_data(self.dc[k], P[ck + ".weight"], self.dr[k - 1] if k > 1 else self.dq1, n, hw, hw, ci, co,
                                   2, 0, wp=self.pk[ck + "b"], stats=st)
            elif dx is not None:
                O.conv3x3_bwd_data(self.dc[0], P[ck + ".weight"], dx, n, hw, hw, ci, co, 2, 0, wp=self.pk[ck + "b"])

    def _g_backward(self, counters=False):
        with O.wgrad_defer(self.wdefer):
            self._g_backward_ops()
            if counters:     # round, G steps, D steps += 1 in the deferred launch; G's completed steps -> dstate[4]
                O.defer_counters(self.dstate[0:3], self.dstate[4:5], 1)

    def _g_backward_ops(self):
        P, G, B = self.G.params, self.G.grads, self.B
        wws = self.wws
        # the Tanh backward also writes conv_blocks.8's bias-gradient partials (CGL_CONV_BIASFUSE; bitwise the
        # weight gradient's column sum over dc3g, one channel-reduction launch fewer)
        bf = self.bpart is not None
        O.act_drop_bwd(self.dimg, self.x3[2 * B:], None, B, 1024, 1, self.dc3g, tanh_y=True,
                       colsum=self.bpart if bf else None)
        db8 = None if bf else G["conv_blocks.8.bias"]
        e6, e2 = self._elided("conv_blocks.6"), self._elided("conv_blocks.2")
        if e6:     # a2 = LeakyReLU(BN(y2)) applied in the operand loads
            O.conv3x3_bwd_weight(self.dc3g, self.y2[B:], G["conv_blocks.8.weight"], db8, B, 32, 32,
                                 64, 1, 1, 0, bn_in=(self.coef["conv_blocks.6"], 1, 2, O.ACT_LEAKY, SLOPE),
                                 ws=wws.get("conv_blocks.8"))
        else:
            O.conv3x3_bwd_weight(self.dc3g, self.a2[B:], G["conv_blocks.8.weight"], db8, B, 32, 32,
                                 64, 1, 1, 0, ws=wws.get("conv_blocks.8"))
        if bf:
            O.colsum_finalize(self.bpart, B * 1024 // 256, 1, G["conv_blocks.8.bias"])
        sm, si = self.g_save["conv_blocks.6"]
        pc6 = self._post_coef("conv_blocks.6")
        kw = dict(post=None if pc6 else self.a2[B:], post_coef=pc6, dgamma=G["conv_blocks.6.weight"],
                  dbeta=G["conv_blocks.6.bias"], slope=SLOPE)
        if self.n1_stats:
            part = self.st_part["conv_blocks.6"]
            O.conv3x3_bwd_data(self.dc3g, P["conv_blocks.8.weight"], self.da2, B, 32, 32, 64, 1, 1, 0,
                               stats=(part, 1, self.y2[B:], kw["post"], sm[1], SLOPE, pc6))
            O.bn2d_bwd_stats(part, self.da2, self.y2[B:], B, 1024, 64, sm[1], si[1], P["conv_blocks.6.weight"],
                             self.dy2, R=128, colsum=self.bcs.get("conv_blocks.6"), **kw)
        else:
            O.conv3x3_bwd_data(self.dc3g, P["conv_blocks.8.weight"], self.da2, B, 32, 32, 64, 1, 1, 0)
            O.bn2d_bwd(self.da2, self.y2[B:], B, 1024, 64, sm[1], si[1], P["conv_blocks.6.weight"], self.dy2, **kw)
        c6 = self.n1_stats and "conv_blocks.6" in self.bcs       # conv_blocks.5's bias from the apply's sums
        db5 = None if c6 else G["conv_blocks.5.bias"]
        if e2:
            O.conv3x3_bwd_weight(self.dy2, self.y1[B:], G["conv_blocks.5.weight"], db5, B, 16, 16,
                                 128, 64, 1, 1, bn_in=(self.coef["conv_blocks.2"], 1, 2, O.ACT_LEAKY, SLOPE),
                                 ws=wws.get("conv_blocks.5"))
        else:
            O.conv3x3_bwd_weight(self.dy2, self.a1[B:], G["conv_blocks.5.weight"], db5, B, 16, 16,
                                 128, 64, 1, 1, ws=wws.get("conv_blocks.5"))
        if c6:
            O.colsum_finalize(self.bcs["conv_blocks.6"], B * 1024 // 256, 64, G["conv_blocks.5.bias"])
        sm, si = self.g_save["conv_blocks.2"]
        st = None
        if self.bst_ok.get("conv_blocks.2"):
            pc2s = self._post_coef("conv_blocks.2")
            st = (self.st_part["conv_blocks.2"], 1, self.y1[B:], None if pc2s else self.a1[B:], sm[1], SLOPE, pc2s)
        O.conv3x3_bwd_data(self.dy2, P["conv_blocks.5.weight"], self.da1, B, 16, 16, 128, 64, 1, 1, wp=self.pk["c5b"],
                           stats=st)
        pc2 = self._post_coef("conv_blocks.2")
        kw = dict(post=None if pc2 else self.a1[B:], post_coef=pc2, dgamma=G["conv_blocks.2.weight"],
                  dbeta=G["conv_blocks.2.bias"], slope=SLOPE)
        c2 = st is not None and "conv_blocks.2" in self.bcs     # conv_blocks.1's bias from the apply's sums
        if st is not None:
            O.bn2d_bwd_stats(self.st_part["conv_blocks.2"], self.da1, self.y1[B:], B, 256, 128, sm[1], si[1],
                             P["conv_blocks.2.weight"], self.dy1, colsum=self.bcs.get("conv_blocks.2"), **kw)
        else:
            O.bn2d_bwd(self.da1, self.y1[B:], B, 256, 128, sm[1], si[1], P["conv_blocks.2.weight"], self.dy1, **kw)
        O.conv3x3_bwd_weight(self.dy1, self.h0[B:], G["conv_blocks.1.weight"], None if c2 else G["conv_blocks.1.bias"],
                             B, 8, 8, 128, 128, 1, 1, ws=wws.get("conv_blocks.1"))
        if c2:
            O.colsum_finalize(self.bcs["conv_blocks.2"], B * 256 // 256, 128, G["conv_blocks.1.bias"])
        O.conv3x3_bwd_data(self.dy1, P["conv_blocks.1.weight"], self.dh0, B, 8, 8, 128, 128, 1, 1, wp=self.pk["c1b"])
        if not self.l1nhwc:
            O.nhwc_to_nchw(self.dh0, self.dh, B, 128, 64)
        self.l1_wgrad()

    # ------------------------------------------------------------------ round
    def phase_a(self, real=None):
        """G forward (Xd, Xg), the local D step, the G loss through the updated D and its gradient
        w.r.t. Xg (capgan.py:215-225, 322-347).  Ends with ``dimg`` = d l_rank / d Xg."""
        with O.stream_cache():     # every op of the phase runs on the current stream
            self._phase_a(real)

    def _round_start(self, real):
        B = self.B
        if self.gen_z:
            if self.graph:
                O.normal_fill_dev(self.z, self.seed, self.dstate[0:1])
            else:
                C.check(C.lib.cgl_normal_fill(ctypes_ptr(self.z), self.z.numel(), self.seed, self.round, 0,
                                              O._s()), "cgl_normal_fill")
        self._short_call = self.short
        if real is not None:
            # an explicit real batch; fewer than B rows = a short batch (padding rows repeat its first row)
            real = real.reshape(-1, 1024)
            nr = real.shape[0]
            if not 1 <= nr <= B:
                raise ValueError(f"real batch of {nr} rows: expected 1 .. {B}")
            O.gather_rows(real, None, 0, nr, 1024, self.x3)
            if nr < B:
                O.gather_rows(real, torch.zeros(B - nr, dtype=torch.int32, device=self.device), 0, B - nr, 1024,
                              self.x3[nr:])
            self._short_call = nr < B or self.short
            if self._short_call:
                self.nv.fill_(nr)
        elif self.data is not None:
            if self.graph:
                O.sample_rows_dev(self.data, B, self.seed + 1 + self.rank, self.dstate[0:1], self.x3,
                                  nv_out=self.nv if self.short else None)
            else:
                self._sample_real()
        self.pk.run()
        self._masks()

    def _phase_a(self, real=None):
        B = self.B
        if self.graph:
            self._sync_dstate()
        # graph rounds: the z draw, the sampler, the weight packing and the Dropout2d masks (independent, all
        # reading the device round counters) go out as ONE launch (cgl_conv_batch_begin / _end)
        with O.launch_batch(self.graph and real is None and self.batch_on):
            self._round_start(real)
        self._g_forward()
        # local D step on [real; Xd]: two forward calls (statistics, masks per call), one backward
        half = 0.5 if self.loss == "mse" else 1.0
        nvd = self.nv if self._short_call else None     # the real call's images (short final batch)
        self._d_forward(self.x3, 2 * B, 2, self.mask_d, nvalid=nvd)
        if self.head_fuse:
            self._head(2 * B, [(B, 1, half, self.lbuf[0:1], nvd), (B, 0, half, self.lbuf[1:2], None)], self.hscr_d,
                       self.flat)
        else:
            with O.launch_batch(self.batch_on):     # the real and fake heads: one launch
                O.adv_loss(self.v[:B], B, 1, self.loss, 1, half, self.lbuf[0:1], self.dv[:B], nvalid=nvd)
                O.adv_loss(self.v[B:2 * B], B, 1, self.loss, 0, half, self.lbuf[1:2], self.dv[B:2 * B])
        self._d_backward(self.x3, 2 * B, 2, self.mask_d, wgrad=True, dx=None, nvalid=nvd)
        self.D.adam(self.lr, self.betas, self.eps, step_dev=self.dstate[2:3] if self.graph else None)
        self.pk.run("D")
        # G loss through the updated D (its D weight gradient is discarded by the reference: skipped)
        self._d_forward(self.x3[2 * B:], B, 1, self.mask_g)
        if self.head_fuse:
            self._head(B, [(B, 1, 1.0, self.lbuf[2:3], None)], self.hscr_g, None)
        else:
            O.adv_loss(self.v[:B], B, 1, self.loss, 1, 1.0, self.lbuf[2:3], self.dv[:B])
        self._d_backward(self.x3[2 * B:], B, 1, self.mask_g, wgrad=False, dx=self.dimg)

    def phase_b(self):
        """Replicated G backward from the (exchanged) image gradient, lambda SGD, Adam G (capgan.py:258-260)."""
        fold = self.graph and self.wdefer and self.cnt_fold
        with O.stream_cache():
            self._g_backward(counters=fold)
            self.G.adam(self.lr, self.betas, self.eps,
                        step_dev=(self.dstate[4:5] if fold else self.dstate[1:2]) if self.graph else None)
            if self.graph:
                if not fold:
                    O.counters_add(self.dstate[0:3], 1)     # round, G steps, D steps (epoch = 1)
                self._dstate_host = (self.round + 1, self.G.step, self.D.step)
        self._lam_step()
        self.round += 1

    def _lam_step(self):
        # optim.SGD([Lambda], lr=0.1) with dF/dLambda = -0.001 (capgan.py:249,259), in the fp32
        # arithmetic of the reference's 0-d tensor (the MLP path's cgl_adam tail does the same)
        if self.weighting != "mean":     # MD-GAN's server has no lambda (MDGAN/MNIST/mdgan.py:203-205)
            self.lam = float(np.float32(self.lam) + np.float32(-0.1) * np.float32(-0.001))

    def run(self, real=None, eager=False):
        """One round with N = 1 (alpha = 1 exactly, capgan.py:247-248).  With graph=True (and the
        round drawing its own real batch) the first round runs eagerly, the second is captured into a
        hipGraph and every round from then on is one replay."""
        if self.n_workers != 1:
            raise RuntimeError("n_workers > 1: use cglgan.exchange.ConvWorkerExchange")
        if not self.graph or eager or real is not None or self.data is None or self.round == 0:
            self.phase_a(real)
            self.phase_b()
            return
        if self._cuda_graph is None:
            self._capture()
        self._sync_dstate()
        self._cuda_graph.replay()
        self._apply_host_delta()

    def run_rounds(self, rounds: int):
        """``rounds`` rounds with N = 1 drawing their own real batches: with graph=True one replay of a graph
        holding ``rounds`` captured rounds back to back (each round reads its per-round values from the device
        counter block the previous one advanced, so this is exactly ``rounds`` calls of ``run()`` without the
        graph-launch boundary between them); otherwise ``rounds`` calls of ``run()``."""
        if rounds <= 0:
            return
        if not self.graph or self.data is None or self.round == 0 or rounds == 1 or self.n_workers != 1:
            for _ in range(rounds):
                self.run()
            return
        g = self._kgraphs.get(rounds)
        if g is None:
            g = self._kgraphs[rounds] = self._capture_rounds(rounds)
        self._sync_dstate()
        g.replay()
        for _ in range(rounds):
            self._apply_host_delta()

    def prepare_rounds(self, rounds: int):
        """Capture the ``rounds``-round graph ahead of its first use (graph=True, N = 1, after the first round)."""
        if self.graph and self.data is not None and self.round > 0 and rounds > 1 and rounds not in self._kgraphs:
            self._kgraphs[rounds] = self._capture_rounds(rounds)

    def _capture_rounds(self, rounds):
        if self._graph_delta is None:
            self._capture()            # (the one-round graph also records the host delta of one round)
        before = self._host_state()
        self._sync_dstate()
        torch.cuda.current_stream().synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            for _ in range(rounds):
                self.phase_a(None)
                self.phase_b()
        # capturing issued nothing: restore the host bookkeeping (run_rounds applies the delta per replayed round)
        self.round, self.G.step, self.D.step = before[0], before[1], before[2]
        self.G.batches.update(before[3])
        self.D.batches.update(before[4])
        self.lam = before[5]
        self._dstate_host = (self.round, self.G.step, self.D.step)
        return g

    # ------------------------------------------------------------------ split round (N > 1)
    def round_a(self, real=None, eager=False):
        """Phase A of a round split at the exchange (N > 1: ConvWorkerExchange / ConvLocalComm issue the
        G-loss all-gather, the lambda weighting and the image-gradient all-reduce between round_a and
        round_b).  With graph=True (and the round drawing its own real batch) every round after the first
        replays phase A and phase B as two hipGraphs captured together; the collectives between them stay
        eager."""
        self._split_graph = (self.graph and not eager and real is None and self.data is not None and
                             self.round > 0)
        if not self._split_graph:
            self.phase_a(real)
            return
        if self._phase_graphs is None:
            self._capture(split=True)
        self._sync_dstate()
        self._phase_graphs[0].replay()

    def round_b(self):
        """Phase B of the split round (after the exchange)."""
        if not self._split_graph:
            self.phase_b()
            return
        self._phase_graphs[1].replay()
        self._apply_host_delta()

    # ------------------------------------------------------------------ graph replay
    def _host_state(self):
        return (self.round, self.G.step, self.D.step, dict(self.G.batches), dict(self.D.batches), self.lam)

    def _sync_dstate(self):
        """dstate must hold (round, G steps, D steps) of the host: rewritten only when the host state
        moved without it (a load_state_dict, a round of another path)."""
        want = (self.round, self.G.step, self.D.step)
        if want != self._dstate_host:
            self.dstate[:3].copy_(torch.tensor(want, dtype=torch.int32))
            self._dstate_host = want

    def _capture(self, split=False):
        before = self._host_state()
        self._sync_dstate()
        torch.cuda.current_stream().synchronize()
        if split:      # phase A and phase B as two graphs (the exchange runs between their replays)
            ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(ga, capture_error_mode="thread_local"):
                self.phase_a(None)
            with torch.cuda.graph(gb, capture_error_mode="thread_local"):
                self.phase_b()
        else:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                self.phase_a(None)
                self.phase_b()
        after = self._host_state()
        # capturing issued nothing: restore the host bookkeeping, remember what one round adds
        self.round, self.G.step, self.D.step = before[0], before[1], before[2]
        self.G.batches.update(before[3])
        self.D.batches.update(before[4])
        self.lam = before[5]
        self._dstate_host = (self.round, self.G.step, self.D.step)
        self._graph_delta = ({k: after[3][k] - before[3][k] for k in before[3]},
                             {k: after[4][k] - before[4][k] for k in before[4]})
        if split:
            self._phase_graphs = (ga, gb)
        else:
            self._cuda_graph = g

    def _apply_host_delta(self):
        gb, db = self._graph_delta
        for k, v in gb.items():
            self.G.batches[k] += v
        for k, v in db.items():
            self.D.batches[k] += v
        self.G.step += 1
        self.D.step += 1
        self._lam_step()
        self.round += 1
        self._dstate_host = (self.round, self.G.step, self.D.step)

    def stats(self):
        l = self.lbuf.cpu()
        half = 0.5 if self.loss == "mse" else 1.0
        return {"round": self.round, "d_real": float(l[0]), "d_fake": float(l[1]),
                "d_loss": float((l[0] + l[1]) * half), "g_loss": float(l[2]), "lambda": self.lam}

    def xd(self):
        return self.x3[self.B:2 * self.B]

    def xg(self):
        return self.x3[2 * self.B:]


def ctypes_ptr(t):
    import ctypes
    return ctypes.c_void_p(t.data_ptr())
