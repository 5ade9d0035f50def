"""Where does the VX=4 GEMM path differ from the VX=1 path?  python tools/diag_vx4.py cin cout res n"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stylemc_amd import _hip, modconv  # noqa: E402

cin, cout, r, n = (int(v) for v in sys.argv[1:5])
torch.manual_seed(0)
W = torch.randn(cout, cin, 3, 3, device="cuda")
P = modconv.PackedConv(W, 1)
x = torch.randn(n, cin, r, r, device="cuda")
ph, nph, th, tw = P.fwd_phases(r, r)
y = torch.empty(n, cout, r, r, device="cuda")
modconv.gemm(x, y, ph, nph, cin, cout, epi=modconv._epilogue(_hip.EPI_STORE))
ref = torch.nn.functional.conv2d(x, W, padding=1)
torch.cuda.synchronize()
d = (y - ref).abs()
print("max err", d.max().item(), "scale", ref.abs().max().item())
bad = (d > 1e-3 * ref.abs().max()).nonzero()
print("bad count", bad.shape[0])
if bad.shape[0]:
    for dim, name in enumerate("ncyx"):
        print(name, torch.unique(bad[:, dim]).tolist()[:40])
