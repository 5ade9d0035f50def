"""Run one modconv GEMM shape repeatedly (for rocprofv3 PMC passes).
    python tools/gemm_one.py KIND R [reps]     KIND in fwd_conv1 fwd_conv0 bwd_conv1 bwd_conv0"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stylemc_amd import _hip, build, modconv  # noqa: E402

kind, r = sys.argv[1], int(sys.argv[2])
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
build.build(verbose=False)
ch = {q: min(32768 // q, 512) for q in [4, 8, 16, 32, 64, 128, 256, 512, 1024]}
n, dev = 4, "cuda"
cin, cout = (ch[r], ch[r]) if kind.endswith("conv1") else (ch[r // 2], ch[r])
up = 1 if kind.endswith("conv1") else 2
h = r // up
W = torch.randn(cout, cin, 3, 3, device=dev)
P = modconv.PackedConv(W, up)
if kind.startswith("fwd"):
    x = torch.randn(n, cin, h, h, device=dev)
    s = torch.randn(n, cin, device=dev)
    ph, nph, th, tw = P.fwd_phases(h, h)
    y = torch.empty(n, cout, th, tw, device=dev)
    run = lambda: modconv.gemm(x, y, ph, nph, cin, cout, s=s, epi=modconv._epilogue(_hip.EPI_STORE))
else:
    t = r if up == 1 else 2 * h + 1
    g = torch.randn(n, cout, t, t, device=dev)
    ph, nph = P.bwd_phases(h, h)
    y = torch.empty(n, cin, h, h, device=dev)
    run = lambda: modconv.gemm(g, y, ph, nph, cout, cin, epi=modconv._epilogue(_hip.EPI_STORE))
for _ in range(reps):
    run()
torch.cuda.synchronize()
print("done", kind, r)
