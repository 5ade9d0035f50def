"""Split-bf16 F(2x2) (smc_set_wino_x3 2) against the fp32 kernel on the same inputs: which tile rows / columns differ."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stylemc_amd import _hip, build, modconv
build.build(verbose=False)
H = _hip; lib = H.load()
dev = "cuda"
for (n, h, w, use_s) in [(4, 128, 128, 1), (4, 256, 256, 0), (4, 256, 256, 1), (4, 1024, 1024, 0), (4, 1024, 1024, 1)]:
    c = 32
    g = torch.Generator().manual_seed(1)
    x = torch.randn(n, c, h, w, generator=g).to(dev)
    sv = (torch.rand(n, c, generator=g) + 0.5).to(dev)
    W_ = (torch.randn(c, c, 3, 3, generator=g) / (3 * c ** 0.5)).to(dev)
    uw = torch.empty(16 * c * c, device=dev)
    H.call("smc_wino_weights_f32", W_.data_ptr(), c, c, 0, uw.data_ptr(), H.stream())
    plain = modconv._epilogue(H.EPI_MODACT, None, None, 0, None, None, "lrelu", 1.0, 1.0, 1e30, None)
    outs = []
    for mode in (0, 2):
        lib.smc_set_wino_x3(mode)
        nb = lib.smc_conv3x3_wino_workspace_size(n, c, c, h, w)
        ws = torch.zeros(max(nb // 4, 1), device=dev)
        y = torch.full((n, c, h, w), float("nan"), device=dev)
        H.call("smc_conv3x3_wino_ws_f32", x.data_ptr(), n, c, h, w, y.data_ptr(), c, uw.data_ptr(), sv.data_ptr() if use_s else None,
               ctypes.byref(plain), ws.data_ptr(), nb, H.stream())
        torch.cuda.synchronize()
        outs.append(y)
    lib.smc_set_wino_x3(0)
    d = (outs[0] - outs[1]).abs()
    bad = d > 1e-4 * outs[0].abs().max()
    print((n, h, w, use_s), "nan", torch.isnan(outs[1]).sum().item(), "bad", bad.sum().item(), "of", bad.numel(), flush=True)
    if bad.any():
        idx = bad.nonzero()
        rows = sorted(set((idx[:, 2] // 2).tolist()))
        print("  bad tile rows (first 20):", rows[:20], "images", sorted(set(idx[:, 0].tolist())), "chans", sorted(set(idx[:, 1].tolist()))[:8])
        cols = sorted(set((idx[:, 3] // 2).tolist()))
        print("  bad tile cols (first 40):", cols[:40])
