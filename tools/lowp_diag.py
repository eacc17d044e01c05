"""Diagnostic: one 16-bit-GEMM round vs the fp64 oracle with and without the operand-rounding
emulation, every checked tensor's relative error (tests/test_gpu_lowp.py's comparison, expanded)."""
import copy
import sys

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, "cgl-gan_amd")
sys.path.insert(0, ".")
from parity_helpers import feed, g_params, inputs, make_pair, oracle_round64, rel, rel_scalar, to_double  # noqa

kind, B, dtype = sys.argv[1], int(sys.argv[2]), sys.argv[3]
DT = {"bf16": torch.bfloat16, "f16": torch.float16, "f32": torch.float32}[dtype]
torch.set_num_threads(8)
srv, workers, step = make_pair(kind, B, gemm_dtype=dtype)
srv64, workers64 = copy.deepcopy(srv), copy.deepcopy(workers)
to_double(srv64, workers64)
emu, wemu = copy.deepcopy(srv64), copy.deepcopy(workers64)
emu.G.lowp = (DT, None)
for w in wemu:
    w.D.lowp = (DT, w.D.spec[-2][1] if w.D.spec[-1][0] == "sigmoid" else w.D.spec[-1][1])
z1, z2, reals = inputs(kind, B, B, 1, seed=11)
feed(step, z1, z2, reals)
step.run()
torch.cuda.synchronize()
st = step.stats()
r64 = oracle_round64(kind, srv64, workers64, z1, z2, reals)
re = oracle_round64(kind, emu, wemu, z1, z2, reals)
out = step.g_output().cpu()
for tag, ref, G, W in (("emu", re, emu.G, wemu), ("exact", r64, srv64.G, workers64)):
    print(tag, "d_loss", rel_scalar(st["d_loss"][0], ref["d_losses"][0]), "g_loss",
          rel_scalar(st["g_loss"], ref["g_losses"][0]), "Xd", rel(out[:B], ref["Xd"].reshape(B, -1)),
          "Xg", rel(out[B:], ref["Xg"].reshape(B, -1)))
    for k, v in step.d_views.items():
        print(tag, "  D", k, rel(v, W[0].D.params[k]))
    p = g_params(G)
    for k, v in step.g_grad_views.items():
        print(tag, "  dG", k, rel(v, p[k].grad))
