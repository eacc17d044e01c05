"""Per-tensor parity report of one conv-GAN round (tests/test_gpu_conv_step.py's check): for every
compared tensor, the HIP error against the fp64 oracle, the fp32 oracle's own error and the ratio
of the HIP error to the 1e-5 relative bound.  Usage: python tools/conv_parity_report.py B loss."""
import os
import sys

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
for p in (ROOT, os.path.join(ROOT, "cgl-gan_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
from test_gpu_conv_step import _err, _run  # noqa: E402


def main(B, loss):
    st, o64, o32, outs = _run(B, loss)
    s, r64, r32, gg, dg = outs[0]
    rows = []
    add = lambda name, h, a, b: rows.append((name, _err(h, a), _err(b, a), float(a.double().norm())))
    add("Xg", st.xg().permute(0, 3, 1, 2), r64["Xg"], r32["Xg"])
    for k, v in r64["g_grads"].items():
        add("G grad " + k, gg[k], v, r32["g_grads"][k])
    for k, v in r64["d_grads"].items():
        add("D grad " + k, dg[k], v, r32["d_grads"][k])
    rows.sort(key=lambda r: -r[1] / max(1e-5 * r[3], 1e-30))
    for name, e, e32, nrm in rows[:12]:
        print(f"B={B} {loss} {name:32s} err {e:.3e} fp32-oracle {e32:.3e} norm {nrm:.3e} "
              f"err/1e-5bound {e / max(1e-5 * nrm, 1e-30):.3f} err/fp32err {e / max(e32, 1e-30):.2f}", flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]), sys.argv[2])
