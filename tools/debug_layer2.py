"""Piecewise check of an up=2 modconv layer: T (transposed conv), U/Y (blur + epilogue), dT (blur adjoint), dx."""
import ctypes
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stylemc_amd import _hip, modconv  # noqa: E402

DEV = "cuda"
n, cin, cout, h = [int(v) for v in (sys.argv[1:5] or [3, 256, 128, 16])]
g = torch.Generator().manual_seed(3)
W = torch.randn(cout, cin, 3, 3, generator=g)
x = torch.randn(n, cin, h, h, generator=g)
s = torch.randn(n, cin, generator=g) * 0.5 + 1
P = modconv.PackedConv(W.to(DEV), 2)
ph, nph, th, tw = P.fwd_phases(h, h)
xd, sd = x.to(DEV), s.to(DEV)
for rep in range(3):
    t = torch.full((n, cout, th, tw), float("nan"), device=DEV)
    modconv.gemm(xd, t, ph, nph, cin, cout, s=sd, epi=modconv._epilogue(_hip.EPI_STORE))
    ref = F.conv_transpose2d((x * s[:, :, None, None]).double(), W.transpose(0, 1).double(), stride=2)
    err = (t.double().cpu() - ref).abs()
    print(f"rep {rep}: T max err {err.max().item():.3e} (scale {ref.abs().max().item():.3e}), nan {int(torch.isnan(t).sum())}")
# backward gather conv alone on a random dT
gT = torch.randn(n, cout, th, tw, generator=g)
phb, nphb = P.bwd_phases(h, h)
dx = torch.empty(n, cin, h, h, device=DEV)
modconv.gemm(gT.to(DEV), dx, phb, nphb, cout, cin, epi=modconv._epilogue(_hip.EPI_STORE))
refb = torch.nn.grad.conv_transpose2d_input if False else None
# adjoint of conv_transpose2d(stride 2) wrt its input = conv2d(gT, W^T layout, stride 2)
refdx = F.conv2d(gT.double(), W.transpose(0, 1).transpose(0, 1).double(), stride=2)
print("bwd gather: max err", (dx.double().cpu() - refdx).abs().max().item(), "scale", refdx.abs().max().item())
