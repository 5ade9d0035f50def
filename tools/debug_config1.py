"""Per-iteration loss terms of the config-1 GPU run vs the reference fixture (tests/golden/config1_direction.npz)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stylemc_amd import networks, synthetic  # noqa: E402
from stylemc_amd.clip_loss import CLIPLoss  # noqa: E402
from stylemc_amd.find_direction import DirectionFinder  # noqa: E402
from stylemc_amd.id_loss import IDLoss  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden"))
from fixture_inputs import LOSS_TEXT  # noqa: E402

DEV = "cuda"
fx = dict(np.load("tests/golden/config1_direction.npz"))
res, bs, n_epochs, seed = (int(v) for v in fx["meta"])
cl = CLIPLoss(DEV, text_features=synthetic.text_direction(*LOSS_TEXT), synthetic_weights=True, seed=4)
idl = IDLoss(device=DEV, weights=None, seed=3)
cfg = synthetic.generator_config(resolution=res)
G = networks.build_generator(cfg, synthetic.generator_state_dict(cfg, seed=0), device=DEV)
f = DirectionFinder(G, torch.from_numpy(fx["styles"]).to(DEV), [(cl, 1.0)], idl, resolution=res, batch_size=bs,
                    n_epochs=n_epochs, seed=seed)
f.load_direction(fx["start"])
for k in range(16):
    last = f.step()
    p = last["parts"].cpu().numpy()
    r = fx["log"][k]
    print(f"it {k + 1:2d} b {last['batch']} clip {p[0] - r[4]:+.2e} id {p[1] - r[5]:+.2e} (id {r[5]:.4f}) l2 {p[3] - r[6]:+.2e}")
cos = torch.nn.functional.cosine_similarity(f.styles_direction.cpu().double().flatten(),
                                            torch.from_numpy(fx["s"]).double().flatten(), dim=0).item()
print("final direction cosine", cos)
