"""Run one Winograd conv shape repeatedly (for rocprofv3 PMC passes).
    python tools/wino_one.py KIND R [reps]     KIND in fwd bwd fwd4 bwd4 (the conv1 of resolution R, batch 4;
                                               fwd4 / bwd4: the F(4x4) kernel)"""
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
f4 = kind.endswith("4")
flip = 0 if kind.startswith("fwd") else 1
uw = P.wino4_weights(flip) if f4 else P.wino_weights(flip)
st = modconv._epilogue(_hip.EPI_STORE)
for _ in range(reps):
    (modconv.wino4 if f4 else modconv.wino)(x, y, uw, c, c, s=s if flip == 0 else None, epi=st)
torch.cuda.synchronize()
print("done", kind, r)
