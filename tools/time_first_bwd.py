"""Which loss net pays the one-time first-backward cost on a fresh box?"""
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402
from stylemc_amd.clip_loss import CLIPLoss  # noqa: E402
from stylemc_amd.id_loss import IDLoss  # noqa: E402
from stylemc_amd import synthetic  # noqa: E402

dev = "cuda"
text = synthetic.text_direction("a", "b")
for bs in (2, 4):
    clip = CLIPLoss(dev, text_features=text, synthetic_weights=True, seed=4)
    idl = IDLoss(device=dev, weights=None, seed=3)
    for name, fn in [("clip", lambda x: clip.per_sample(torch.nn.functional.interpolate(x.detach(), 224), torch.nn.functional.interpolate(x, 224)).sum()),
                     ("id", lambda x: idl.per_sample(x, x.detach()).sum())]:
        for rep in range(2):
            x = torch.randn(bs, 3, 256, 256, device=dev, requires_grad=True)
            torch.cuda.synchronize(); t0 = time.time()
            l = fn(x); torch.cuda.synchronize(); t1 = time.time()
            g, = torch.autograd.grad(l, x); torch.cuda.synchronize(); t2 = time.time()
            print(f"bs{bs} {name} rep{rep}: fwd {t1 - t0:.2f}s bwd {t2 - t1:.2f}s", flush=True)
