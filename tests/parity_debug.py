"""Diagnostic (not collected by pytest): per-tensor error of the HIP round and of the fp32
oracle, each against the same oracle run in float64.  Separates real kernel errors from the
conditioning of the reference computation itself.

    python tests/parity_debug.py capgan 64
"""
import copy
import sys

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, "cgl-gan_amd")
sys.path.insert(0, ".")

from parity_helpers import feed, inputs, make_pair, oracle_round  # noqa: E402


def to_double(srv, workers):
    def conv_net(n):
        nets = [n.trunk] + list(n.heads) if hasattr(n, "trunk") else [n]
        for net in nets:
            for k in list(net.params):
                net.params[k] = net.params[k].detach().double().requires_grad_(True)
            for k in list(net.buffers):
                if net.buffers[k].dtype == torch.float32:
                    net.buffers[k] = net.buffers[k].double()
    conv_net(srv.G)
    srv.opt.params = srv.G.parameters()
    srv.opt.m = [m.double() for m in srv.opt.m]
    srv.opt.v = [v.double() for v in srv.opt.v]
    srv.beta = srv.beta.double()
    for w in workers:
        conv_net(w.D)
        w.opt.params = w.D.parameters()
        w.opt.m = [m.double() for m in w.opt.m]
        w.opt.v = [v.double() for v in w.opt.v]


def params_of(G):
    nets = [G.trunk] + list(G.heads) if hasattr(G, "trunk") else [G]
    out = {}
    for n in nets:
        out.update(n.params)
    return out


def rel(a, b):
    a = a.detach().double().cpu().flatten()
    b = b.detach().double().cpu().flatten()
    return float((a - b).norm() / max(float(b.norm()), 1e-300))


def g_intermediates64(G, D, z2, loss="ce"):
    """fp64 autograd pass of the Xg forward call with every Linear output / activation kept."""
    import torch.nn.functional as F
    nets = [G.trunk] + list(G.heads) if hasattr(G, "trunk") else [G]
    h = z2.double()
    ys, acts = [], []
    for net in nets:
        spec = net.spec
        for i, ent in enumerate(spec):
            if ent[0] == "linear":
                h = F.linear(h, net.params[ent[1] + ".weight"].detach(), net.params[ent[1] + ".bias"].detach())
                h.requires_grad_(True) if not h.requires_grad else None
                h.retain_grad()
                ys.append(h)
            elif ent[0] == "bn":
                k = ent[1]
                h = F.batch_norm(h, None, None, net.params[k + ".weight"].detach(), net.params[k + ".bias"].detach(),
                                 True, 0.1, 0.8)
            elif ent[0] == "leaky":
                h = F.leaky_relu(h, 0.2)
                h.retain_grad()
                acts.append(h)
            elif ent[0] == "tanh":
                h = torch.tanh(h)
    out = h
    logits = D.forward(out)
    t = torch.ones(out.shape[0], dtype=torch.long)
    l = F.cross_entropy(logits, t)
    l.backward()
    return ys, acts


def main(kind="capgan", B=64):
    torch.set_num_threads(1)
    srv, workers, step = make_pair(kind, B)
    srv64, workers64 = copy.deepcopy(srv), copy.deepcopy(workers)
    to_double(srv64, workers64)
    G_before64 = copy.deepcopy(srv64.G)
    z1, z2, reals = inputs(kind, B, B, 1, seed=7)
    feed(step, z1, z2, reals)
    step.run()
    torch.cuda.synchronize()
    r32 = oracle_round(kind, srv, workers, z1, z2, reals)
    torch.set_default_dtype(torch.float64)
    r64 = oracle_round(kind, srv64, workers64, z1.double(), z2.double(), [r.double() for r in reals])
    torch.set_default_dtype(torch.float32)
    st = step.stats()
    print(f"{kind} B={B}")
    print(f"  d_loss  gpu-vs64 {abs(st['d_loss'][0]-float(r64['d_losses'][0]))/abs(float(r64['d_losses'][0])):.2e}"
          f"  cpu32-vs64 {abs(float(r32['d_losses'][0])-float(r64['d_losses'][0]))/abs(float(r64['d_losses'][0])):.2e}")
    if kind in ("capgan", "mixg1", "mixg1x"):
        torch.set_default_dtype(torch.float64)
        ys, acts = g_intermediates64(G_before64, workers64[0].D, z2)
        torch.set_default_dtype(torch.float32)
        L = len(ys)
        print("  backward intermediates (gpu vs fp64):")
        print(f"    dYL (pre-tanh grad)    {rel(step.internal(2).view(B, -1), ys[L - 1].grad):.2e}")
        for l in range(L - 1):
            gG = step.internal(32 + l).view(B, -1)
            print(f"    gG[{l}] (dL/dy_{l})       {rel(gG, ys[l].grad):.2e}   |ref| {float(ys[l].grad.norm()):.2e}")
            if step.gm.bn[l]:
                gdA = step.internal(16 + l).view(B, -1)
                print(f"    gdA[{l}] (dL/da_{l})      {rel(gdA, acts[l].grad):.2e}")
                ga = step.internal(48 + l).view(2 * B, -1)[B:]
                print(f"    gact[{l}] (a_{l})          {rel(ga, acts[l].detach()):.2e}")
            go = step.internal(64 + l).view(2 * B, -1)[B:]
            print(f"    gout[{l}] (y_{l})          {rel(go, ys[l].detach()):.2e}")
            if step.gm.bn[l]:
                # host recomputation of BN backward from the GPU's own inputs (fp64)
                y = go.double().cpu()
                post = step.internal(48 + l).view(2 * B, -1)[B:].double().cpu()
                dA = step.internal(16 + l).view(B, -1).double().cpu()
                mean_g = step.internal(80 + l).view(2, -1)[1].double().cpu()
                inv_g = step.internal(96 + l).view(2, -1)[1].double().cpu()
                mean_t = y.mean(0)
                inv_t = 1.0 / torch.sqrt(y.var(0, unbiased=False) + 0.8)
                dy = torch.where(post > 0, dA, dA * 0.2)
                gam = G_before64.trunk.params if hasattr(G_before64, "trunk") else G_before64.params
                key = step.gm.bn_keys[l] + ".weight"
                if key not in gam:
                    gam = G_before64.heads[0].params
                w = gam[key].detach()
                S = dy.sum(0)
                Dd = ((y - mean_t) * dy).sum(0)
                dz = (dy - S / B - (y - mean_t) * Dd * inv_t ** 2 / B) * inv_t * w
                print(f"      saved mean err {rel(mean_g, mean_t):.2e}  invstd err {rel(inv_g, inv_t):.2e}  "
                      f"|mean|/std {float(mean_t.abs().mean() / (y.std(0).mean())):.2e}")
                ref_post = acts[l].detach().cpu()
                flips = ((post > 0) != (ref_post > 0))
                print(f"      mask flips {int(flips.sum())}; min |post| at flips "
                      f"{float(post[flips].abs().min()) if flips.any() else 0:.3e}; ref there "
                      f"{float(ref_post[flips].abs().min()) if flips.any() else 0:.3e}; "
                      f"exact zeros gpu {int((post == 0).sum())} ref {int((ref_post == 0).sum())}")
                print(f"      host BN-bwd from GPU inputs vs fp64 ref {rel(dz, ys[l].grad):.2e}; "
                      f"GPU gG vs host {rel(step.internal(32 + l).view(B, -1), dz):.2e}; "
                      f"|dy|/|dz| {float(dy.norm() / dz.norm()):.2e}")
    p32, p64 = params_of(srv.G), params_of(srv64.G)
    print("  G grads:                 gpu-vs-64   cpu32-vs-64  gpu-vs-cpu32   |g64|")
    for k, v in step.g_grad_views.items():
        print(f"    {k:22s} {rel(v, p64[k].grad):.2e}    {rel(p32[k].grad, p64[k].grad):.2e}    "
              f"{rel(v, p32[k].grad):.2e}    {float(p64[k].grad.norm()):.2e}")
    print("  G params:")
    for k, v in step.g_views.items():
        print(f"    {k:22s} {rel(v, p64[k]):.2e}    {rel(p32[k], p64[k]):.2e}    {rel(v, p32[k]):.2e}")
    print("  D params:")
    for k, v in step.d_views.items():
        print(f"    {k:22s} {rel(v, workers64[0].D.params[k]):.2e}    "
              f"{rel(workers[0].D.params[k], workers64[0].D.params[k]):.2e}    {rel(v, workers[0].D.params[k]):.2e}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "capgan", int(sys.argv[2]) if len(sys.argv) > 2 else 64)
