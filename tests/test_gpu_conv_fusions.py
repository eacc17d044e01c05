"""Two conv-round fusions that must leave every tensor of the round bitwise unchanged (model/lsgan.py:13-22,
78-80), eager and graph-replayed, at B = 8 and the benchmarked B = 256:
  * CGL_CONV_POSTCOEF: the G BatchNorm2d backward takes LeakyReLU'(a) from the sign of the forward's own
    fmaf(y, scale, shift) (cgl_bn2d_bwd / cgl_bn2d_bwd_stats post_coef: the coef the forward finalize kept)
    instead of reading the activation a -- the forward wrote a = LeakyReLU(that value);
  * CGL_CONV_DFOLD: in the G-loss pass, D's inner BatchNorm2d layers are applied in the next conv's operand
    load (bn_in, cgl_eltwise's fmaf) instead of an apply pass -- nothing else reads their output there;
    CGL_CONV_DFOLD_STEP (opt-in): in the D step too, the weight gradients applying them in their loads;
  * CGL_CONV_BATCH: the graph round's start (weight packing, Dropout2d masks, z draw, real-batch sampler) as one
    launch (cgl_conv_batch_begin / _end);
  * CGL_CONV_N1STATS: conv_blocks.6's backward partials written by the Conv2d(64, 1) input gradient itself
    (cgl_conv3x3_bwd_data_stats, 128-row chunks) instead of a channel reduction over the stored gradient;
  * CGL_CONV_BIASFUSE: conv_blocks.8's bias-gradient partials written by the Tanh backward (cgl_act_drop_bwd_colsum)
    instead of the weight gradient's column sum over the stored gradient;
  * CGL_CONV_C1FUSE: D's Conv2d(1, 16) weight gradient in the D step applies its block's LeakyReLU + Dropout2d
    backward in its loads (cgl_conv3x3_bwd_weight_actdrop) instead of after an act_drop_bwd pass;
  * CGL_CONV_ELIDE: a folded G BatchNorm's activation (a1 / a2) is not stored at all -- the G backward's weight
    gradients apply the BatchNorm in their operand loads (cgl_conv3x3_bwd_weight_bnin) and every LeakyReLU'
    comes from the kept scale / shift (with the same fold mask on both sides);
  * CGL_CONV_WDEFER: a backward pass's weight-gradient split reductions (and Conv2d(1, 16)'s finish) deferred to
    one launch at the end of the pass (cgl_conv_wgrad_defer_begin / _end).
  * CGL_CONV_BNBCOL: the G BatchNorm backward applies also write their output's column sums (the producing convs'
    bias gradients, cgl_bn2d_bwd_stats colsum_part) instead of the weight gradient's own pass.
  * CGL_CONV_L1NHWC: G's Linear(100, 8192) gathers its weight rows in NHWC feature order (with the bias packed in
    that order) and writes the NHWC activation directly, instead of the NCHW output + a transpose launch.
  * CGL_CONV_CNTFOLD: graph rounds advance the device round / step counters in the G backward's deferred launch
    (cgl_conv_wgrad_defer_counters) instead of a cgl_counters_add launch; G Adam reads the snapshot.
  * CGL_CONV_HEADBN: D's last BatchNorm (model.14) applied in the fused head's loads instead of by cgl_eltwise.
  * CGL_CONV_HEADFUSE: the discriminator head (adv_layer forward, the loss head(s), adv_layer's input gradient) as
    one launch per pass (cgl_dense1_head_nhwc), its batch-mean losses reduced by the last workgroup."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _step(B, graph, data, env):
    from cglgan.conv_step import ConvGanStep
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        st = ConvGanStep(B, seed=21, data=data, graph=graph)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    st.init_default(5, 6)
    return st


CASES = [("CGL_CONV_POSTCOEF", 8, False, "2"), ("CGL_CONV_POSTCOEF", 256, False, "0"),
         ("CGL_CONV_POSTCOEF", 256, True, "2"), ("CGL_CONV_DFOLD", 8, False, "2"), ("CGL_CONV_DFOLD", 256, True, "2"),
         ("CGL_CONV_DFOLD_STEP", 8, False, "2"), ("CGL_CONV_DFOLD_STEP", 256, True, "2"),
         ("CGL_CONV_BATCH", 8, True, "3"), ("CGL_CONV_BATCH", 256, True, "3"),
         ("CGL_CONV_ELIDE", 8, False, "3"), ("CGL_CONV_ELIDE", 256, False, "3"), ("CGL_CONV_ELIDE", 256, True, "3"),
         ("CGL_CONV_ELIDE", 256, True, "2"), ("CGL_CONV_N1STATS", 8, False, "3"),
         ("CGL_CONV_N1STATS", 256, True, "3"), ("CGL_CONV_N1STATS", 256, False, "0"),
         ("CGL_CONV_BIASFUSE", 8, False, "3"), ("CGL_CONV_BIASFUSE", 256, True, "3"),
         ("CGL_CONV_C1FUSE", 8, False, "3"), ("CGL_CONV_C1FUSE", 256, True, "3"),
         ("CGL_CONV_HEADFUSE", 8, False, "3"), ("CGL_CONV_HEADFUSE", 256, True, "3"),
         ("CGL_CONV_WDEFER", 8, False, "3"), ("CGL_CONV_WDEFER", 256, True, "3"), ("CGL_CONV_WDEFER", 256, False, "0"),
         ("CGL_CONV_HEADBN", 8, False, "3"), ("CGL_CONV_HEADBN", 256, True, "3"),
         ("CGL_CONV_BNBCOL", 8, False, "3"), ("CGL_CONV_BNBCOL", 256, True, "3"), ("CGL_CONV_BNBCOL", 256, False, "0"),
         ("CGL_CONV_L1NHWC", 8, False, "3"), ("CGL_CONV_L1NHWC", 256, True, "3"),
         ("CGL_CONV_CNTFOLD", 8, True, "3"), ("CGL_CONV_CNTFOLD", 256, True, "3")]


@pytest.mark.parametrize("var,B,graph,fold", CASES)
def test_conv_round_fusion_bitwise(var, B, graph, fold):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        data = torch.rand(4 * B + 3, 1024, device="cuda", generator=torch.Generator("cuda").manual_seed(3)) * 2 - 1
        a = _step(B, graph, data, {var: "1", "CGL_CONV_BNFOLD": fold})
        b = _step(B, graph, data, {var: "0", "CGL_CONV_BNFOLD": fold})
        for _ in range(3):
            a.run()
            b.run()
        torch.cuda.synchronize()
    if var == "CGL_CONV_POSTCOEF":
        assert a.post_coef_on and not b.post_coef_on
        assert {"conv_blocks.2", "conv_blocks.6"} <= a.coef_kept
    elif var == "CGL_CONV_DFOLD":
        assert a.d_fold and not b.d_fold
    elif var == "CGL_CONV_BATCH":
        assert a.batch_on and not b.batch_on
    elif var == "CGL_CONV_N1STATS":
        assert a.n1_stats and not b.n1_stats
    elif var == "CGL_CONV_BIASFUSE":
        assert a.bpart is not None and b.bpart is None
    elif var == "CGL_CONV_C1FUSE":
        assert a.c1_fuse and not b.c1_fuse
    elif var == "CGL_CONV_HEADFUSE":
        assert a.head_fuse and not b.head_fuse
        assert torch.equal(a.v, b.v) and torch.equal(a.dv, b.dv) and torch.equal(a.dr[3], b.dr[3])
    elif var == "CGL_CONV_WDEFER":
        assert a.wdefer and not b.wdefer
    elif var == "CGL_CONV_BNBCOL":
        assert a.bnb_col and not b.bnb_col and (B < 256 or len(a.bcs) == 2)
    elif var == "CGL_CONV_L1NHWC":
        assert a.l1nhwc and not b.l1nhwc
        assert torch.equal(a.h0, b.h0)
    elif var == "CGL_CONV_CNTFOLD":
        assert a.cnt_fold and not b.cnt_fold
        assert torch.equal(a.dstate[:4], b.dstate[:4]) and a.dstate[:3].tolist() == [3, 3, 3]
        assert a.dstate[4].item() == 2      # the G steps completed before the third round's G Adam
    elif var == "CGL_CONV_HEADBN":
        assert a.head_bn and not b.head_bn
        assert torch.equal(a.v, b.v) and torch.equal(a.dv, b.dv) and torch.equal(a.dr[3], b.dr[3])
    elif var == "CGL_CONV_DFOLD_STEP":
        assert a.d_fold_step and not b.d_fold_step and a._d_folded and not b._d_folded
    else:
        assert a.elide_on and not b.elide_on and a.bn_fold == b.bn_fold
        for k in ("a1", "a2"):
            assert torch.allclose(a.g_act(k), b.g_act(k), rtol=1e-6, atol=1e-6), k
    for name in ("p", "g", "m", "v"):
        assert torch.equal(getattr(a.G, name), getattr(b.G, name)), ("G", name)
        assert torch.equal(getattr(a.D, name), getattr(b.D, name)), ("D", name)
    for k in a.D.running:
        assert torch.equal(a.D.running[k], b.D.running[k]), k
    assert torch.equal(a.x3, b.x3) and torch.equal(a.lbuf, b.lbuf)
    assert torch.equal(a.dy1, b.dy1) and torch.equal(a.dy2, b.dy2)


@pytest.mark.parametrize("loss,B", [("mse", 8), ("bce", 8), ("bce", 256)])
def test_head_fuse_short_batch(loss, B):
    """The fused head over a pass with a short final real batch (3 real rows): its nvalid call, both losses."""
    from cglgan.conv_step import ConvGanStep
    s = torch.cuda.Stream()
    outs = []
    with torch.cuda.stream(s):
        data = torch.rand(2 * B + 3, 1024, device="cuda", generator=torch.Generator("cuda").manual_seed(4)) * 2 - 1
        for on in ("1", "0"):
            old = os.environ.get("CGL_CONV_HEADFUSE")
            os.environ["CGL_CONV_HEADFUSE"] = on
            try:
                st = ConvGanStep(B, loss=loss, seed=31, data=data, graph=True)
            finally:
                if old is None:
                    os.environ.pop("CGL_CONV_HEADFUSE", None)
                else:
                    os.environ["CGL_CONV_HEADFUSE"] = old
            st.init_default(7, 8)
            lb = []
            for _ in range(4):            # rounds 0, 1 full, round 2 the short batch (3 rows), round 3 full
                st.run()
                lb.append(st.lbuf.clone())
            torch.cuda.synchronize()
            outs.append((st, lb))
    (a, la), (b, lb) = outs
    assert a.head_fuse and not b.head_fuse and a.short
    assert all(torch.equal(x, y) for x, y in zip(la, lb))
    assert torch.equal(a.D.p, b.D.p) and torch.equal(a.G.p, b.G.p) and torch.equal(a.D.g, b.D.g)
    assert torch.equal(a.v, b.v) and torch.equal(a.dv, b.dv) and torch.equal(a.dr[3], b.dr[3])
