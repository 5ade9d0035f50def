"""CPU restatement of StyleMC's S-space synthesis driver (TEST ORACLE ONLY).

  block_forward   <- utils.py:13-53   (per-block forward from S codes, widths trimmed by `shapes`)
  generate_image  <- utils.py:161-216 (block loop up to until_k; blending branches omitted: they are
                     only taken with use_blending=True, which find_direction never sets)
  get_temp_shapes <- utils.py:100-120 (records affine widths and replaces each affine by Identity)
  split_ws        <- utils.py:77-87
  get_styles      <- utils.py:123-158 (W -> packed S [n, 26, 512])
"""
import torch

from . import ops

N_STYLE_CHANNELS = 26                                     # find_direction.py:39
S_TRAINABLE_SPACE_CHANNELS = [2, 3, 5, 6, 8, 9, 11, 12]   # find_direction.py:41


def block_forward(block, x, img, ws, shapes, force_fp32=True, fused_modconv=None, **layer_kwargs):
    assert ws.ndim == 3 and ws.shape[1] == block.num_conv + block.num_torgb
    rows = list(ws.unbind(dim=1))
    if fused_modconv is None:
        fused_modconv = not block.training   # fp32 everywhere in the oracle
    if block.in_channels == 0:
        x = block.const.to(torch.float32).unsqueeze(0).repeat([ws.shape[0], 1, 1, 1])
        x = block.conv1(x, rows[0][..., :shapes[0]], fused_modconv=fused_modconv, **layer_kwargs)
        rgb_row = rows[1]
    else:
        assert x.shape[1:] == (block.in_channels, block.resolution // 2, block.resolution // 2)
        x = x.to(torch.float32)
        x = block.conv0(x, rows[0][..., :shapes[0]], fused_modconv=fused_modconv, **layer_kwargs)
        x = block.conv1(x, rows[1][..., :shapes[1]], fused_modconv=fused_modconv, **layer_kwargs)
        rgb_row = rows[2]
    if img is not None:
        img = ops.upsample2d(img, block.resample_filter)
    y = block.torgb(x, rgb_row[..., :shapes[2]], fused_modconv=fused_modconv).to(torch.float32)
    img = img.add_(y) if img is not None else y
    return x, img


def generate_image(G, until_k, styles, temp_shapes, noise_mode="const", device=None):
    x = img = None
    xs = []
    row = 0
    for k, res in enumerate(G.synthesis.block_resolutions):
        if k > until_k:
            continue
        block = getattr(G.synthesis, f"b{res}")
        width = 2 if res == 4 else 3
        x, img = block_forward(block, x, img, styles[:, row:row + width, :], temp_shapes[k], noise_mode=noise_mode)
        row += width
        xs.append(x)
    return xs, img


def get_temp_shapes(G):
    shapes = []
    for res in G.synthesis.block_resolutions:
        block = getattr(G.synthesis, f"b{res}")
        names = ["conv1", "conv1", "torgb"] if res == 4 else ["conv0", "conv1", "torgb"]
        shapes.append(tuple(getattr(block, n).affine.weight.shape[0] for n in names))
        for n in set(names):
            getattr(block, n).affine = torch.nn.Identity()
    return shapes


def split_ws(G, ws):
    out = []
    idx = 0
    for res in G.synthesis.block_resolutions:
        block = getattr(G.synthesis, f"b{res}")
        out.append(ws.to(torch.float32).narrow(1, idx, block.num_conv + block.num_torgb))
        idx += block.num_conv
    return out


@torch.no_grad()
def get_styles(G, ws):
    """W [n, num_ws, 512] -> S [n, 26, 512] (zero padded); mutates G like the reference."""
    block_ws = split_ws(G, ws)
    styles = torch.zeros(ws.shape[0], N_STYLE_CHANNELS, 512, device=ws.device)
    row = 0
    shapes = []
    for res, cur in zip(G.synthesis.block_resolutions, block_ws):
        block = getattr(G.synthesis, f"b{res}")
        layers = [block.conv1, block.torgb] if res == 4 else [block.conv0, block.conv1, block.torgb]
        widths = [l.affine.weight.shape[0] for l in layers]
        shapes.append((widths[0], widths[0], widths[1]) if res == 4 else tuple(widths))
        for j, layer in enumerate(layers):
            styles[:, row + j, :widths[j]] = layer.affine(cur[:, j, :])
            layer.affine = torch.nn.Identity()
        row += len(layers)
    return styles, shapes
