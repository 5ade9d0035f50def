"""Locate IR-SE50 HIP/fp64 differences: truncated networks (stem + first k units + an output Linear)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from torch import nn  # noqa: E402

from stylemc_amd import build, irse_hip, synthetic  # noqa: E402
from stylemc_amd.id_loss.model_irse import Backbone  # noqa: E402


class Trunc(nn.Module):
    def __init__(self, full, k):
        super().__init__()
        self.input_layer = full.input_layer
        self.body = nn.Sequential(*list(full.body)[:k])
        last = full.body[k - 1].res_layer[3]
        depth = last.out_channels
        hw = 112
        for u in list(full.body)[:k]:
            hw //= u.res_layer[3].stride[0]
        g = torch.Generator().manual_seed(k)
        lin = nn.Linear(depth * hw * hw, 512)
        lin.weight.data = torch.randn(512, depth * hw * hw, generator=g) / (depth * hw * hw) ** 0.5
        bn2 = nn.BatchNorm2d(depth).eval()
        bn1 = nn.BatchNorm1d(512).eval()
        self.output_layer = nn.Sequential(bn2, nn.Dropout(0.0), nn.Flatten(), lin, bn1)

    def forward(self, x):
        x = self.output_layer(self.body(self.input_layer(x)))
        return x


def main():
    build.build(verbose=False)
    full = Backbone(112, 50, "ir_se", 0.6).eval()
    full.load_state_dict(synthetic.seeded_state_dict(full, seed=3))
    x = torch.randn(2, 3, 112, 112, generator=torch.Generator().manual_seed(0))
    cot = torch.randn(2, 512, generator=torch.Generator().manual_seed(1))
    for k in [int(a) for a in (sys.argv[1:] or ["1", "2", "3", "4", "5", "8", "21", "22", "24"])]:
        t = Trunc(full, k).eval().requires_grad_(False)
        pk = irse_hip._Packed(t, "cuda")
        xr = x.double().requires_grad_(True)
        yr = t.double()(xr)
        (dxr,) = torch.autograd.grad(yr, xr, cot.double())
        t.float()
        mod = irse_hip.HipIRSE50()
        mod._packed = pk
        xg = x.cuda().requires_grad_(True)
        yg = irse_hip._IrseFn.apply(xg, mod, None)
        (dxg,) = torch.autograd.grad(yg, xg, cot.cuda())
        ey = ((yg.cpu().double() - yr).abs().max() / yr.abs().max()).item()
        d = (dxg.cpu().double() - dxr).abs()
        ed = (d.max() / dxr.abs().max()).item()
        idx = torch.nonzero(d == d.max())[0].tolist()
        # error by border/interior
        inner = d[:, :, 1:-1, 1:-1].max().item() / dxr.abs().max().item()
        print(f"k={k:2d}: y rel {ey:.2e}  dx rel {ed:.2e} at {idx}  interior {inner:.2e}  "
              f"per-channel max rel {[round((d[:, c].max() / dxr.abs().max()).item(), 6) for c in range(3)]}",
              flush=True)


if __name__ == "__main__":
    main()
