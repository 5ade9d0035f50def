"""Debug one SynthesisLayer forward/backward vs the oracle, piece by piece.  python tools/debug_layer.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_ops import _pair_layers  # noqa: E402

DEV = "cuda"
cin, cout, res, up, n = [int(v) for v in (sys.argv[1:6] or [256, 128, 32, 2, 1])]
mode = sys.argv[6] if len(sys.argv) > 6 else "none"
o, p = _pair_layers(cin, cout, res, up, clamp=256.0)
gen = torch.Generator().manual_seed(3)
x = torch.randn(n, cin, res // up, res // up, generator=gen)
s = torch.randn(n, cin, generator=gen) * 0.5 + 1
cot = torch.randn(n, cout, res, res, generator=gen)
xr, sr = x.clone().requires_grad_(True), s.clone().requires_grad_(True)
yr = o(xr, sr, noise_mode=mode, fused_modconv=True)
dxr, dsr = torch.autograd.grad((yr * cot).sum(), [xr, sr])
xg, sg = x.to(DEV).requires_grad_(True), s.to(DEV).requires_grad_(True)
yg = p(xg, sg, noise_mode=mode)
dxg, dsg = torch.autograd.grad((yg * cot.to(DEV)).sum(), [xg, sg])
for name, a, b in (("y", yg, yr), ("dx", dxg, dxr), ("ds", dsg, dsr)):
    a = a.detach().double().cpu()
    b = b.detach().double()
    err = (a - b).abs()
    sc = b.abs().max().item()
    print(f"{name}: max err {err.max().item():.3e} scale {sc:.3e}, >1e-4*scale: {int((err > 1e-4 * sc).sum())}")
    if name == "dx":
        bad = (err > 1e-4 * sc).nonzero()
        print("  first bad idx", bad[:8].tolist())
        print("  per-channel bad counts (top)", torch.bincount(bad[:, 1], minlength=cin).topk(5))
        print("  spatial bad", torch.bincount(bad[:, 2] * 100 + bad[:, 3]).nonzero().flatten()[:20].tolist())
