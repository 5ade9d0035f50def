"""Seeded inputs and output summaries shared by make_golden.py (which runs the reference) and the tests
(which run the oracle / the HIP path): large inputs are regenerated from seeds instead of being stored."""
import torch

from stylemc_amd import synthetic

LOSS_TEXT = ("a photo of a face of a feminine woman with no makeup", "a photo of a face of a masculine man")


def loss_inputs(n=2, res=512, seed=21):
    """Edited / original image pair in about [-1.3, 1.3] (so unprocess clamps), S codes and a delta."""
    g = torch.Generator().manual_seed(seed)
    orig = (torch.randn(n, 3, res, res, generator=g) * 0.6).clamp(-1.3, 1.3)
    img = orig + 0.08 * torch.randn(n, 3, res, res, generator=g)
    styles = synthetic.synthetic_styles(n, seed=seed)
    delta = torch.randn(1, 8, 512, generator=g) * 0.05
    return img, orig, styles, delta


def block_sums(t, k=8):
    """k x k block sums of an image-shaped gradient (the stored summary of d loss / d img)."""
    return torch.nn.functional.avg_pool2d(t.double(), k) * (k * k)


def probes(t, n=8, seed=99):
    """n seeded random projections of a tensor (fp64)."""
    g = torch.Generator().manual_seed(seed)
    P = torch.randn(n, t.numel(), generator=g, dtype=torch.float64)
    return P @ t.detach().cpu().double().flatten()
