"""Diagnostic: IR-SE50 input gradient with split-bf16 vs exact-fp32 direct GEMMs, against fp64 (max and norm error,
cosine, how many PReLU pre-activations change sign between the two forms).

    python tools/irse_x3_diag.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from stylemc_amd import build, modconv, irse_hip, synthetic
    from stylemc_amd.id_loss.model_irse import Backbone
    build.build(verbose=False)
    ref = Backbone(112, 50, "ir_se", 0.6).eval()
    ref.load_state_dict(synthetic.seeded_state_dict(ref, seed=3))
    ref = ref.requires_grad_(False).double()
    for n in (1, 4, 8):
        gen = torch.Generator().manual_seed(n)
        x = torch.randn(n, 3, 112, 112, generator=gen)
        cot = torch.randn(n, 512, generator=gen)
        xr = x.double().requires_grad_(True)
        (dxr,) = torch.autograd.grad(ref(xr), xr, cot.double())
        scale = dxr.abs().max().item()
        res = {}
        for x3 in (False, True):
            modconv.X3 = x3
            hip = irse_hip.build_irse50(seed=3, device="cuda")
            xg = x.cuda().requires_grad_(True)
            yg = hip(xg)
            (dxg,) = torch.autograd.grad(yg, xg, cot.cuda())
            d = dxg.cpu().double()
            e_max = (d - dxr).abs().max().item() / scale
            e_norm = ((d - dxr).norm() / dxr.norm()).item()
            cos = torch.nn.functional.cosine_similarity(d.flatten(), dxr.flatten(), dim=0).item()
            res[x3] = d
            print(f"n={n} {'x3  ' if x3 else 'fp32'}: max err {e_max:.3e}  norm err {e_norm:.3e}  cos {cos:.8f}",
                  flush=True)
        diff = (res[True] - res[False]).abs()
        print(f"n={n} x3 vs fp32: max {diff.max().item() / scale:.3e}, elements beyond 1e-4 of max: "
              f"{int((diff > 1e-4 * scale).sum())} of {diff.numel()}", flush=True)


if __name__ == "__main__":
    main()
