"""IR-SE50 forward features + input gradient of fixed seeded faces (n = 1, 4, 8), saved for bit-comparing library
variants (SMC_HIP_LIB).    python tools/irse_dump.py OUT.npz"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from stylemc_amd import _hip, irse_hip
    _hip.load()
    net = irse_hip.build_irse50(None, seed=3, device="cuda")
    out = {}
    g = torch.Generator().manual_seed(0)
    for n in (1, 4, 8):
        x = torch.randn(n, 3, 112, 112, generator=g).cuda().requires_grad_(True)
        f = net(x, n_grad=max(1, n // 2))
        w = torch.randn(f.shape, generator=g).cuda()
        (dx,) = torch.autograd.grad((f * w).sum(), x)
        out[f"f{n}"] = f.detach().cpu().numpy()
        out[f"dx{n}"] = dx.cpu().numpy()
    np.savez(sys.argv[1], **out)
    print("saved", sys.argv[1])


if __name__ == "__main__":
    main()
