"""Diagnostic: gather-conv GEMM vs torch conv2d on the GPU over a grid of shapes/splits."""
import itertools
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stylemc_amd import _hip, modconv  # noqa: E402

torch.backends.cudnn.allow_tf32 = False
dev = "cuda"
bad = 0
for cin, cout, n, res, split in itertools.product([16, 32, 128], [16, 32, 64, 128], [1, 2], [8, 64], ["", "1", "4"]):
    if split:
        os.environ["SMC_FORCE_SPLIT"] = split
    else:
        os.environ.pop("SMC_FORCE_SPLIT", None)
    g = torch.Generator().manual_seed(0)
    W = torch.randn(cout, cin, 3, 3, generator=g).to(dev)
    x = torch.randn(n, cin, res, res, generator=g).to(dev)
    ref = F.conv2d(x, W, padding=1)
    P = modconv.PackedConv(W, 1)
    y = torch.empty_like(ref)
    ph, nph, _, _ = P.fwd_phases(res, res)
    modconv.gemm(x, y, ph, nph, cin, cout, epi=modconv._epilogue(_hip.EPI_STORE))
    torch.cuda.synchronize()
    err = (y - ref).abs().max().item() / ref.abs().max().item()
    flag = "BAD" if err > 1e-5 else ""
    bad += bool(flag)
    print(f"cin={cin:4d} cout={cout:4d} n={n} res={res:3d} split={split or 'auto':4s} err={err:.2e} {flag}")
print("bad:", bad)

# transposed stride-2 conv (4 polyphase phases; fused path unless SMC_NO_CONVT_FUSION is set)
bad_t = 0
for cin, cout, n, h, split in itertools.product([16, 64, 128], [16, 32, 64, 128], [1, 2], [4, 33], ["", "1", "3"]):
    if split:
        os.environ["SMC_FORCE_SPLIT"] = split
    else:
        os.environ.pop("SMC_FORCE_SPLIT", None)
    g = torch.Generator().manual_seed(1)
    W = torch.randn(cout, cin, 3, 3, generator=g).to(dev)
    x = torch.randn(n, cin, h, h, generator=g).to(dev)
    s = (torch.randn(n, cin, generator=g) * 0.5 + 1).to(dev)
    ref = F.conv_transpose2d(x * s[:, :, None, None], W.transpose(0, 1), stride=2)
    P = modconv.PackedConv(W, 2)
    ph, nph, th, tw = P.fwd_phases(h, h)
    y = torch.full((n, cout, th, tw), float("nan"), device=dev)
    modconv.gemm(x, y, ph, nph, cin, cout, s=s, epi=modconv._epilogue(_hip.EPI_STORE))
    torch.cuda.synchronize()
    err = ((y - ref).abs().max() / ref.abs().max()).item()
    flag = "BAD" if not (err <= 1e-5) else ""
    bad_t += bool(flag)
    print(f"convT cin={cin:4d} cout={cout:4d} n={n} h={h:3d} split={split or 'auto':4s} err={err:.2e} {flag}")
os.environ.pop("SMC_FORCE_SPLIT", None)
print("bad convT:", bad_t)
