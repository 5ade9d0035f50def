"""Run one Winograd conv shape repeatedly (for rocprofv3 PMC passes).
    python tools/wino_one.py KIND R [reps]     KIND in fwd bwd (the conv1 of resolution R, batch 4)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stylemc_amd import _hip, build, modconv  # noqa: E402

kind, r = sys.argv[1], int(sys.argv[2])
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
build.build(verbose=False)
n, dev = 4, "cuda"
c = min(32768 // r, 512)
W = torch.randn(c, c, 3, 3, device=dev) / (3 * c ** 0.5)
P = modconv.PackedConv(W, 1)
x = torch.randn(n, c, r, r, device=dev)
s = torch.rand(n, c, device=dev) + 0.5
y = torch.empty_like(x)
uw = P.wino_weights(0 if kind == "fwd" else 1)
st = modconv._epilogue(_hip.EPI_STORE)
for _ in range(reps):
    modconv.wino(x, y, uw, c, c, s=s if kind == "fwd" else None, epi=st)
torch.cuda.synchronize()
print("done", kind, r)
