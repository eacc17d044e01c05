#!/usr/bin/env python3
"""Which single op breaks torch.cuda.graph capture?  Each case runs in its own subprocess (a crash in one
does not hide the others):  python tools/capture_probe.py  -> one line per case (ok / rc).

Round 5 adds the r04 segfault's own pattern (tests/test_gpu_cglgan_modules.py, an eager G -> D -> CE ->
backward step whose outputs -- and so its autograd graph -- stay alive across the side-stream warm-up and
the capture) in four forms: the library's modules or plain torch modules (nn.Linear / BatchNorm1d /
LeakyReLU / Tanh, no libcglgan call at all), eager graph alive or deleted before the capture:
alive_hip, del_hip, alive_torch, del_torch."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = ["linear_fwd", "linear_fwd_act", "linear_bwd_data", "linear_bwd_weight", "bn1d_fwd", "bn1d_bwd", "act_fwd",
         "gen_fwd", "disc_fwd", "gen_fwd_bwd", "torch_only", "g_sum_none", "gd_sum_keep", "gd_ce_keep", "gd_ce_none",
         "d_ce_none", "g_bn_only_none", "test_exact", "test_b64", "test_noeager", "test_nosnap",
         "alive_torch", "del_torch", "alive_hip", "del_hip"]


def torch_models():
    """model/mnist_model.py's Generator / Discriminator as plain torch modules (reference structure)."""
    import torch.nn as nn

    def block(i, o, bn=True):
        layers = [nn.Linear(i, o)] + ([nn.BatchNorm1d(o, 0.8)] if bn else []) + [nn.LeakyReLU(0.2)]
        return layers
    G = nn.Sequential(*block(100, 128, False), *block(128, 256), *block(256, 512), *block(512, 1024),
                      nn.Linear(1024, 784), nn.Tanh())
    D = nn.Sequential(nn.Linear(784, 512), nn.LeakyReLU(0.2), nn.Linear(512, 256), nn.LeakyReLU(0.2),
                      nn.Linear(256, 2))
    return G, D


def run_alive(name):
    """The r04 test's flow; ``alive_*`` keeps the eager step's outputs (its autograd graph) across the capture."""
    sys.path.insert(0, os.path.join(ROOT, "cgl-gan_amd"))
    import torch
    torch.manual_seed(5)
    if name.endswith("_hip"):
        from cglgan import model as CM
        G, D = CM.Generator((1, 28, 28)).cuda(), CM.Discriminator((1, 28, 28)).cuda()
        fwd = lambda z: D(G(z))
    else:
        G, D = torch_models()
        G, D = G.cuda(), D.cuda()
        fwd = lambda z: D(G(z).view(z.shape[0], -1))
    z = torch.randn(128, 100, device="cuda")
    params = list(G.parameters()) + list(D.parameters())

    def step():
        out = fwd(z)
        loss = torch.nn.functional.cross_entropy(out, torch.ones(out.shape[0], dtype=torch.long, device="cuda"))
        loss.backward()
        return out, loss
    for q in params:
        q.grad = None
    keep = step()
    if name.startswith("del_"):
        del keep
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            for q in params:
                q.grad = None
            step()
    torch.cuda.current_stream().wait_stream(s)
    for q in params:
        q.grad = None
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    g.replay()
    torch.cuda.synchronize()
    print("CASE-OK", name, flush=True)


def run_test_like(name):
    """tests/test_gpu_cglgan_modules.py::test_module_forward_backward_graph_capture_bitwise, with knobs."""
    import copy
    sys.path.insert(0, os.path.join(ROOT, "cgl-gan_amd"))
    import torch
    from cglgan import model as CM
    torch.manual_seed(5)
    B = 64 if name == "test_b64" else 128
    G = CM.Generator((1, 28, 28)).cuda()
    D = CM.Discriminator((1, 28, 28)).cuda()
    z = torch.randn(B, 100, device="cuda")
    snaps = None if name == "test_nosnap" else [copy.deepcopy(m.state_dict()) for m in (G, D)]
    params = list(G.parameters()) + list(D.parameters())

    def step():
        out = D(G(z))
        loss = torch.nn.functional.cross_entropy(out, torch.ones(out.shape[0], dtype=torch.long, device="cuda"))
        loss.backward()
        return out, loss
    if name != "test_noeager":
        for q in params:
            q.grad = None
        step()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            for q in params:
                q.grad = None
            step()
    torch.cuda.current_stream().wait_stream(s)
    for q in params:
        q.grad = None
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    if snaps:
        for m, sd in zip((G, D), snaps):
            m.load_state_dict(sd)
    g.replay()
    torch.cuda.synchronize()
    print("CASE-OK", name, flush=True)


def run_case(name):
    if name.startswith("test_"):
        return run_test_like(name)
    if name.startswith("alive_") or name.startswith("del_"):
        return run_alive(name)
    sys.path.insert(0, os.path.join(ROOT, "cgl-gan_amd"))
    import torch
    from cglgan import model as CM
    import cglgan._lib as C
    dev = "cuda"
    torch.manual_seed(0)
    M, K, N = 128, 100, 256
    x = torch.randn(M, K, device=dev)
    w = torch.randn(N, K, device=dev)
    b = torch.randn(N, device=dev)
    y = torch.empty(M, N, device=dev)
    ws = torch.empty(C.lib.cgl_op_workspace_bytes(), dtype=torch.uint8, device=dev)
    p = lambda t: CM._p(t)
    G = CM.Generator((1, 28, 28)).to(dev)
    D = CM.Discriminator((1, 28, 28)).to(dev)
    z = torch.randn(64, 100, device=dev)
    dy = torch.randn(M, N, device=dev)
    dx = torch.empty(M, K, device=dev)
    dw = torch.empty(N, K, device=dev)
    db = torch.empty(N, device=dev)
    g1 = torch.ones(N, device=dev)
    b1 = torch.zeros(N, device=dev)
    rm, rv = torch.zeros(N, device=dev), torch.ones(N, device=dev)
    sm, si = torch.empty(N, device=dev), torch.empty(N, device=dev)
    xb = torch.randn(M, N, device=dev)

    def op():
        s = CM._s()
        if name == "linear_fwd":
            C.check(C.lib.cgl_linear_fwd(p(x), p(w), p(b), p(y), M, N, K, 0, 0.2, p(ws), ws.numel(), s))
        elif name == "linear_fwd_act":
            C.check(C.lib.cgl_linear_fwd(p(x), p(w), p(b), p(y), M, N, K, 1, 0.2, p(ws), ws.numel(), s))
        elif name == "linear_bwd_data":
            C.check(C.lib.cgl_linear_bwd_data(p(dy), p(w), p(dx), M, N, K, p(ws), ws.numel(), s))
        elif name == "linear_bwd_weight":
            C.check(C.lib.cgl_linear_bwd_weight(p(dy), p(x), p(dw), p(db), M, N, K, p(ws), ws.numel(), s))
        elif name == "bn1d_fwd":
            C.check(C.lib.cgl_bn1d_fwd(p(xb), M, N, N, p(g1), p(b1), 0.8, 0.1, p(rm), p(rv), 1, 1, 0.2, p(y), p(sm),
                                       p(si), p(ws), ws.numel(), s))
        elif name == "bn1d_bwd":
            C.check(C.lib.cgl_bn1d_bwd(p(dy), p(y), p(xb), M, N, p(sm), p(si), p(g1), 1, 0.2, p(dx), p(db), p(b1),
                                       p(ws), ws.numel(), s))
        elif name == "act_fwd":
            C.check(C.lib.cgl_act_fwd(p(xb), xb.numel(), 1, 0.2, p(y), s))
        elif name == "gen_fwd":
            G(z)
        elif name == "disc_fwd":
            D(torch.randn(64, 784, device=dev))
        elif name == "gen_fwd_bwd":
            G(z).sum().backward()
        elif name == "torch_only":
            torch.mm(x, w.t()).relu().sum()
        elif name in ("g_sum_none",):
            G(z).sum().backward()
        elif name == "gd_sum_keep":
            D(G(z)).sum().backward()
        elif name in ("gd_ce_keep", "gd_ce_none"):
            out = D(G(z))
            torch.nn.functional.cross_entropy(out, torch.ones(out.shape[0], dtype=torch.long, device=dev)).backward()
        elif name == "d_ce_none":
            out = D(xd)
            torch.nn.functional.cross_entropy(out, torch.ones(out.shape[0], dtype=torch.long, device=dev)).backward()
        elif name == "g_bn_only_none":
            Gb(z).sum().backward()
    xd = torch.randn(64, 784, device=dev, requires_grad=True)
    Gb = torch.nn.Sequential(torch.nn.Linear(100, 256), torch.nn.BatchNorm1d(256, 0.8), torch.nn.LeakyReLU(0.2)).to(dev)
    Gb_mod = Gb
    class _W(torch.nn.Module):
        def forward(self, t):
            return CM.run_sequential(Gb_mod, t)
    Gb = _W()
    none = name.endswith("_none")

    def clear():
        if none:
            for q in list(G.parameters()) + list(D.parameters()) + list(Gb_mod.parameters()) + [xd]:
                q.grad = None
    if name == "bn1d_bwd":
        C.check(C.lib.cgl_bn1d_fwd(p(xb), M, N, N, p(g1), p(b1), 0.8, 0.1, p(rm), p(rv), 1, 1, 0.2, p(y), p(sm),
                                   p(si), p(ws), ws.numel(), CM._s()))
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            clear()
            op()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    clear()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        op()
    g.replay()
    torch.cuda.synchronize()
    print("CASE-OK", name, flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        run_case(sys.argv[1])
        sys.exit(0)
    for c in CASES:
        r = subprocess.run([sys.executable, "-u", __file__, c], capture_output=True, text=True, timeout=120)
        ok = r.returncode == 0 and "CASE-OK" in r.stdout
        tail = "" if ok else (r.stdout + r.stderr).strip().splitlines()[-3:]
        print(f"{c:20s} {'ok' if ok else 'FAIL rc=' + str(r.returncode)} {tail}", flush=True)
