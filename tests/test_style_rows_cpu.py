"""Host logic of the synthesis' S-row gather (utils._gather_rows), no GPU: every row a layer reads, the trainable
rows as one [T, N, 512] block (delta added in one op), the ToRGB rows times their weight_gain -- checked against
plain per-row slicing, the form block_forward uses (utils.py:13-53 of the reference)."""
import torch

from stylemc_amd import networks, synthetic, utils


def _gen(res=64):
    cfg = synthetic.generator_config(resolution=res, channel_base=2048, channel_max=128)
    return networks.build_generator(cfg, device="cpu")


def test_gather_rows_matches_slices():
    G = _gen()
    shapes = utils.get_temp_shapes(G)
    n = 3
    styles = torch.randn(n, 26, 512)
    until_k = len(G.synthesis.block_resolutions) - 1
    T = [2, 3, 5, 6, 8, 9, 11, 12]
    T = [r for r in T if r < 2 + 3 * until_k]  # rows this 64-px generator has
    gains = {1: 0.5, 4: 0.25, 7: 0.125}
    out, block = utils._gather_rows(G, until_k, styles, shapes, full=set(T), lead=T, gains=gains)
    row = 0
    for k, res in enumerate(G.synthesis.block_resolutions):
        sh = shapes[k]
        widths = (sh[0], sh[2]) if res == 4 else tuple(sh)
        for j, w in enumerate(widths):
            r = row + j
            want = styles[:, r, :(512 if r in T else w)]
            if r in gains:
                want = want * gains[r]   # float32 x python float: the layer's own product
            assert out[r].is_contiguous()
            assert torch.equal(out[r], want), r
        row += len(widths)
    assert block.shape == (len(T), n, 512)
    assert torch.equal(block, torch.stack([styles[:, r] for r in T]))
    for j, r in enumerate(T):  # the block and the dict share storage
        assert out[r].data_ptr() == block[j].data_ptr()


def test_gather_rows_lead_needs_every_row():
    G = _gen()
    shapes = utils.get_temp_shapes(G)
    styles = torch.randn(2, 26, 512)
    # until_k = 1: rows 0..4 only, so a lead naming row 5 falls back to the per-row form (no block)
    out, block = utils._gather_rows(G, 1, styles, shapes, full={2, 5}, lead=[2, 5])
    assert block is None
    assert torch.equal(out[2], styles[:, 2])
    assert 5 not in out


def test_delta_block_gradient_is_per_row_sum():
    """The one-op delta add (generate_image_rows) differentiates like the per-row form it replaced."""
    n, T = 4, 8
    block = torch.randn(T, n, 512)
    delta = torch.randn(1, T, 512, requires_grad=True)
    rows = (block + delta.reshape(-1, T, 512).transpose(0, 1)).unbind(0)
    gs = [torch.randn(n, 512) for _ in range(T)]
    (g1,) = torch.autograd.grad(sum((r * g).sum() for r, g in zip(rows, gs)), delta)
    d2 = delta.detach().clone().requires_grad_(True)
    rows2 = [block[j] + d2[:, j] for j in range(T)]
    (g2,) = torch.autograd.grad(sum((r * g).sum() for r, g in zip(rows2, gs)), d2)
    assert torch.allclose(g1, g2, rtol=0, atol=1e-5)
    for j in range(T):
        assert torch.equal(rows[j], rows2[j])
