"""Diagnostic: IR-SE50 input gradient with split-bf16 vs exact-fp32 direct GEMMs, against fp64 (max and norm error,
cosine), and the conditioning of that gradient itself: the fp64 reference re-run on inputs perturbed by one fp32
rounding (x * (1 + 2^-24 r), r ~ N(0, 1)) -- how far the EXACT gradient moves when the input moves by the error any
fp32 implementation makes.  If that move is as large as the x3 / fp32 errors, the errors are the input gradient's
own discontinuity (a PReLU / SE-ReLU pre-activation within rounding of its kink takes the other branch), not lost
product bits.

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
        for k in range(3):   # the exact gradient at inputs one fp32 rounding away
            r = torch.randn(x.shape, generator=gen, dtype=torch.float64)
            xp = (x.double() * (1 + 2.0 ** -24 * r)).requires_grad_(True)
            (dxp,) = torch.autograd.grad(ref(xp), xp, cot.double())
            print(f"n={n} fp64 at x(1 + 2^-24 r) #{k}: max move {(dxp - dxr).abs().max().item() / scale:.3e}  "
                  f"norm move {((dxp - dxr).norm() / dxr.norm()).item():.3e}  elements beyond 1e-4 of max: "
                  f"{int(((dxp - dxr).abs() > 1e-4 * scale).sum())}", flush=True)
        res = {}
        for x3 in (False, True):
            irse_hip.X3 = x3
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
