"""Batch invariance of every piece of the find_direction step on the GPU (the exact N-rank parity of SURVEY 8(e)).

A data-parallel shard computes its images in a smaller batch than the single process does.  Under
``_hip.plan_batch(plan, local)`` every batch-dependent launch decision is made for the full batch, so each image must
come out BIT FOR BIT as in the full batch: the synthesis forward and its per-image style gradient, the CLIP ViT
embedding and image gradient, the IR-SE50 features and input gradient, the loss heads' row reductions, and finally the
step's per-image gradient rows.  Also: the row-reduction kernels against fp64.
"""
import pytest
import torch

from tests import dist_gpu_worker as W

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _rel(a, b):
    return ((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-30)).item()


def test_row_ops_vs_fp64():
    from stylemc_amd import rowops
    g = torch.Generator().manual_seed(3)
    a = torch.randn(7, 512, generator=g)
    b = torch.randn(7, 512, generator=g)
    t = torch.nn.functional.normalize(torch.randn(1, 512, generator=g), dim=1)
    ref = (a.double() * b.double()).sum(1)
    assert _rel(rowops.row_dot(a.to(DEV), b.to(DEV)).cpu(), ref) < 1e-6
    assert _rel(rowops.row_dot(a.to(DEV), t.to(DEV)).cpu(), (a.double() * t.double()).sum(1)) < 1e-6
    # l2_normalize forward / backward vs autograd in fp64
    x = a.double().requires_grad_(True)
    y = x / x.norm(dim=1, keepdim=True)
    gy = b.double()
    (gx,) = torch.autograd.grad(y, x, gy)
    xd = a.to(DEV).requires_grad_(True)
    yd = rowops.l2_normalize(xd)
    (gxd,) = torch.autograd.grad(yd, xd, b.to(DEV))
    assert _rel(yd.detach().cpu(), y.detach()) < 1e-6 and _rel(gxd.cpu(), gx) < 1e-5
    # the directional CLIP head: loss and d loss / d e vs autograd of the reference formula in fp64
    e = a.double().requires_grad_(True)
    src = b.double()
    f = e - src
    f = f / f.norm(dim=1, keepdim=True)
    loss = 1 - torch.nn.functional.cosine_similarity(f, t.double())
    (ge,) = torch.autograd.grad(loss.sum(), e)
    ld, gd = rowops.direction_head(a.to(DEV), b.to(DEV), t.to(DEV))
    assert _rel(ld.cpu(), loss.detach()) < 1e-5 and _rel(gd.cpu(), ge) < 1e-5


def test_row_ops_rows_independent_of_batch():
    from stylemc_amd import rowops
    g = torch.Generator().manual_seed(4)
    a = torch.randn(8, 512, generator=g).to(DEV)
    b = torch.randn(8, 512, generator=g).to(DEV)
    t = torch.nn.functional.normalize(torch.randn(1, 512, generator=g), dim=1).to(DEV)
    full = rowops.row_dot(a, b)
    l8, g8 = rowops.direction_head(a, b, t)
    for lo, hi in ((0, 1), (2, 4), (5, 8)):
        assert torch.equal(rowops.row_dot(a[lo:hi], b[lo:hi]), full[lo:hi])
        l, gr = rowops.direction_head(a[lo:hi], b[lo:hi], t)
        assert torch.equal(l, l8[lo:hi]) and torch.equal(gr, g8[lo:hi])


def test_step_pieces_batch_invariant():
    """Each network of the step, and the step's per-image rows, at batch 4 against the same images as shards of 2
    and 1 under the planning scope.  Every mismatch is listed (a failure names the piece that depends on the batch)."""
    from stylemc_amd import _hip, synthetic, utils
    from stylemc_amd.find_direction import DirectionFinder, initial_delta
    G, clip, idl, shapes = W.problem(DEV)
    cl = clip[0][0]
    styles = synthetic.synthetic_styles(4, seed=5).to(DEV)
    delta = initial_delta(0, 0.01).to(DEV)
    bad = []

    f = DirectionFinder(G, styles, clip, idl, resolution=W.RES, batch_size=4, global_batch=4, n_epochs=4, seed=1,
                        init_delta=initial_delta(0, 0.01), temp_shapes=shapes)

    def synth(st):
        d = delta.expand(st.shape[0], -1, -1).clone().requires_grad_(True)
        img = utils.generate_image_rows(G, f.until_k, st, shapes, "const", delta=d)
        (gd,) = torch.autograd.grad(img, d, torch.ones_like(img))
        return img.detach(), gd

    def vit(x, n_grad):
        x = x.detach().requires_grad_(True)
        e = cl.visual(x, n_grad=n_grad)
        (gx,) = torch.autograd.grad(e[:n_grad], x, torch.ones_like(e[:n_grad]))
        return e.detach(), gx[:n_grad]

    def irse(x, n_grad):
        x = x.detach().requires_grad_(True)
        f = idl.facenet(x, n_grad=n_grad)
        (gx,) = torch.autograd.grad(f[:n_grad], x, torch.ones_like(f[:n_grad]))
        return f.detach(), gx[:n_grad]

    img4, gd4 = synth(styles)
    gen = torch.Generator().manual_seed(9)
    x224 = torch.randn(8, 3, 224, 224, generator=gen).to(DEV)
    x112 = torch.randn(8, 3, 112, 112, generator=gen).to(DEV)
    e8, gv8 = vit(x224, 4)
    f8, gi8 = irse(x112, 4)
    rows4 = f._local_terms(styles, 4)
    for lo, hi in ((0, 2), (2, 4), (3, 4)):
        n = hi - lo
        with _hip.plan_batch(4, n):
            img, gd = synth(styles[lo:hi])
            # the loss networks see [edited; original] pairs of the shard: rows lo..hi of each half
            idx = torch.cat([torch.arange(lo, hi), torch.arange(4 + lo, 4 + hi)]).to(DEV)
            e, gv = vit(x224[idx], n)
            fi, gi = irse(x112[idx], n)
            rows = f._local_terms(styles[lo:hi], 4)
        for name, got, ref in (("synthesis image", img, img4[lo:hi]), ("synthesis style grad", gd, gd4[lo:hi]),
                               ("ViT embedding", e, e8[idx]), ("ViT image grad", gv, gv8[lo:hi]),
                               ("IR-SE50 features", fi, f8[idx]), ("IR-SE50 input grad", gi, gi8[lo:hi]),
                               ("step rows", rows, rows4[lo:hi])):
            if not torch.equal(got, ref):
                bad.append((name, (lo, hi), _rel(got, ref)))
    assert not bad, bad
