"""Debug aid: first G-forward layer whose output differs between the LDS-staged GEMM loop and the
register loop (same state, same explicit inputs); usage: python tools/gl_debug.py B kind."""
import os
import subprocess
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def child(gl, B, kind, out):
    os.environ["CGL_GEMM_GL"] = gl
    sys.path[:0] = [ROOT, os.path.join(ROOT, "cgl-gan_amd"), os.path.join(ROOT, "tests")]
    import torch
    from parity_helpers import feed, inputs, make_pair
    srv, workers, step = make_pair(kind, B)
    z1, z2, reals = inputs(kind, B, B, 1, 5)
    feed(step, z1, z2, reals)
    step.run()
    torch.cuda.synchronize()
    res = {f"gout{l}": step.internal(64 + l).clone().cpu() for l in range(step.gm.n_layers)}
    res.update({f"P{j}": step.internal(112 + j).clone().cpu() for j in range(step.dm.n_layers - 1)})
    torch.save(res, out)


if __name__ == "__main__":
    if len(sys.argv) > 4:
        child(sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4])
        sys.exit(0)
    B, kind = sys.argv[1], sys.argv[2]
    for gl in ("0", "1"):
        subprocess.run([sys.executable, __file__, gl, B, kind, f"/tmp/gl{gl}.pt"], check=True)
    import torch
    a, b = torch.load("/tmp/gl0.pt"), torch.load("/tmp/gl1.pt")
    for k in a:
        d = (a[k] - b[k]).abs()
        print(k, "max diff", float(d.max()), "at", int(d.argmax()), "numel", a[k].numel(), flush=True)
