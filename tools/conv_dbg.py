"""Debug helper: one conv3x3 op vs torch (fp64, CPU), printing where the mismatches are."""
import sys
import torch
import torch.nn.functional as F
sys.path.insert(0, "cgl-gan_amd")
from cglgan import conv_ops as O

n, h, w, cin, cout, stride, up, act = [int(x) for x in sys.argv[1:9]]
g = torch.Generator().manual_seed(0)
x = torch.randn(n, cin, h, w, generator=g, dtype=torch.float64)
W = torch.randn(cout, cin, 3, 3, generator=g, dtype=torch.float64) * 0.1
b = torch.randn(cout, generator=g, dtype=torch.float64)
xi = F.interpolate(x, scale_factor=2, mode="nearest") if up else x
ref = F.conv2d(xi, W, b, stride, 1)
ho, wo = ref.shape[2], ref.shape[3]
xd = x.permute(0, 2, 3, 1).contiguous().float().cuda()
y = torch.full((n, ho, wo, cout), 777.0, device="cuda")
O.conv3x3_fwd(xd, W.float().cuda(), b.float().cuda(), y, n, h, w, cin, cout, stride, up, act, slope=float(sys.argv[9]) if len(sys.argv) > 9 else 0.2)
torch.cuda.synchronize()
got = y.double().cpu().permute(0, 3, 1, 2)
err = (got - ref).abs()
bad = (err > 1e-3 * ref.abs().max())
print("bad", int(bad.sum()), "of", bad.numel(), "unwritten", int((got == 777.0).sum()))
idx = bad.nonzero()[:20]
for i in idx.tolist():
    print(i, float(got[tuple(i)]), float(ref[tuple(i)]))
# pattern per (oy parity, ox parity) and per channel block
if bad.any():
    print("per oy%2,ox%2:", [[int(bad[:, :, a::2, c::2].sum()) for c in (0, 1)] for a in (0, 1)])
    print("per img:", [int(bad[i].sum()) for i in range(n)])
    print("per ch32:", [int(bad[:, c:c + 32].sum()) for c in range(0, cout, 32)])
