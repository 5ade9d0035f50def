"""The fused loss nodes (clip_loss._DirectionHead, find_direction._LossTotal) against autograd through the reference's
op-by-op formulas (clip_loss.py:7-34 direction loss; find_direction.py:318-330 loss composition): same forward
values, gradients equal to autograd's in fp64 to 1e-12 and within a few ulp in fp32."""
import torch
import torch.nn.functional as F

from stylemc_amd import clip_loss
from stylemc_amd import find_direction as FD


def _ref_head(e, src, t):
    f = e - src
    f = f / f.norm(dim=1, keepdim=True)
    return 1 - F.cosine_similarity(f, t)


def _head_case(dtype):
    g = torch.Generator().manual_seed(3)
    e = torch.randn(6, 512, generator=g, dtype=dtype)
    src = torch.randn(6, 512, generator=g, dtype=dtype)
    t = torch.randn(1, 512, generator=g, dtype=dtype)
    t = t / t.norm(dim=1, keepdim=True)
    w = torch.rand(6, generator=g, dtype=dtype)
    e1 = e.clone().requires_grad_(True)
    e2 = e.clone().requires_grad_(True)
    y1 = clip_loss._DirectionHead.apply(e1, src, t)
    y2 = _ref_head(e2, src, t)
    (y1 * w).sum().backward()
    (y2 * w).sum().backward()
    return y1, y2, e1.grad, e2.grad


def test_direction_head_fp64():
    y1, y2, g1, g2 = _head_case(torch.float64)
    assert torch.equal(y1, y2)
    assert (g1 - g2).abs().max().item() <= 1e-12 * g2.abs().max().item()


def test_direction_head_fp32():
    y1, y2, g1, g2 = _head_case(torch.float32)
    assert torch.equal(y1, y2)
    assert (g1 - g2).abs().max().item() <= 2e-6 * g2.abs().max().item()


def test_direction_loss_switch():
    g = torch.Generator().manual_seed(4)
    e = torch.randn(3, 64, generator=g).requires_grad_(True)
    src = torch.randn(3, 64, generator=g)
    t = torch.nn.functional.normalize(torch.randn(1, 64, generator=g), dim=1)
    assert clip_loss.direction_loss(e, src, t).grad_fn.__class__.__name__.startswith("_DirectionHead")
    src_g = src.clone().requires_grad_(True)   # a differentiable source embedding keeps autograd's graph
    assert not clip_loss.direction_loss(e, src_g, t).grad_fn.__class__.__name__.startswith("_DirectionHead")


def test_loss_total_matches_autograd():
    g = torch.Generator().manual_seed(5)
    n, T = 4, 8
    for dtype, tol in ((torch.float64, 1e-12), (torch.float32, 2e-6)):
        idt = torch.rand(n, generator=g, dtype=dtype)
        clt = torch.rand(n, generator=g, dtype=dtype)
        d = torch.randn(T, 1, 512, generator=g, dtype=dtype) * 0.01
        sT = torch.randn(T, n, 512, generator=g, dtype=dtype)
        c_id, c_clip, c_l2, denom = 0.6, 1.0, 0.1, n
        l2_den = float(denom * T * 512)
        a = [x.clone().requires_grad_(True) for x in (idt, clt, d)]
        b = [x.clone().requires_grad_(True) for x in (idt, clt, d)]
        tot, parts = FD._LossTotal.apply(a[0], a[1], a[2], sT, c_id, c_clip, c_l2, l2_den, float(denom))
        l2_sum = ((sT + b[2]) - sT).square().sum()
        id_part = c_id * b[0].sum() / denom
        clip_part = c_clip * b[1].sum() / denom
        l2_part = c_l2 * l2_sum / (denom * T * 512)
        ref = id_part + clip_part + l2_part
        assert torch.equal(tot, ref)
        assert torch.equal(parts, torch.stack([clip_part, id_part, torch.zeros_like(l2_part), l2_part]).detach())
        ga = torch.autograd.grad(tot, a)
        gb = torch.autograd.grad(ref, b)
        for x, y in zip(ga, gb):
            assert (x - y).abs().max().item() <= tol * y.abs().max().item()
