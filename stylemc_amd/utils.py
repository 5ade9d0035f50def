"""S-space synthesis driver -- drop-in for the reference's utils.py hot-path helpers.

  block_forward   (utils.py:13-53)   per-block forward from S codes; widths trimmed by `shapes`
  generate_image  (utils.py:161-216) block loop up to `until_k`; `device` is optional here (the
                                     reference's find_direction.py:309,312 omits it -> TypeError there)
  get_temp_shapes (utils.py:100-120) style widths per block; replaces each affine by Identity
  split_ws        (utils.py:77-87), get_styles (utils.py:123-158), get_mean_std (utils.py:90-97)
The feature-blending branches of generate_image (use_blending, cv2 masks) are out of scope
 and raise NotImplementedError.
"""
import torch

from .torch_utils.ops import upfirdn2d

N_STYLE_CHANNELS = 26
S_TRAINABLE_SPACE_CHANNELS = [2, 3, 5, 6, 8, 9, 11, 12]
S_NON_TRAINABLE_SPACE_CHANNELS = [0, 1, 4, 7, 10, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25]


def block_forward(self, x, img, ws, shapes, force_fp32=False, fused_modconv=None, **layer_kwargs):
    assert ws.ndim == 3 and ws.shape[1] == self.num_conv + self.num_torgb and ws.shape[2] == self.w_dim
    w_iter = iter(ws.unbind(dim=1))
    if fused_modconv is None:
        fused_modconv = not self.training
    if self.in_channels == 0:
        x = self.const.to(torch.float32).unsqueeze(0).repeat([ws.shape[0], 1, 1, 1])
        x = self.conv1(x, next(w_iter)[..., :shapes[0]], fused_modconv=fused_modconv, **layer_kwargs)
    else:
        assert x.shape[1:] == (self.in_channels, self.resolution // 2, self.resolution // 2)
        x = x.to(torch.float32)
        x = self.conv0(x, next(w_iter)[..., :shapes[0]], fused_modconv=fused_modconv, **layer_kwargs)
        x = self.conv1(x, next(w_iter)[..., :shapes[1]], fused_modconv=fused_modconv, **layer_kwargs)
    if img is not None:
        assert img.shape[1:] == (self.img_channels, self.resolution // 2, self.resolution // 2)
        img = upfirdn2d.upsample2d(img, self.resample_filter)
    if self.is_last or self.architecture == "skip":
        y = self.torgb(x, next(w_iter)[..., :shapes[2]], fused_modconv=fused_modconv)
        y = y.to(dtype=torch.float32, memory_format=torch.contiguous_format)
        img = img.add_(y) if img is not None else y
    return x, img


def generate_image(G, until_k, styles, temp_shapes, noise_mode="const", device=None, use_blending=False,
                   xs_original=None, masks_dict=None):
    if use_blending or xs_original is not None:
        raise NotImplementedError("feature blending (deeplab masks) is outside the find_direction hot path")
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


_GATHER_IDX = {}


def _gather_rows(G, until_k, styles, temp_shapes, full=(), lead=(), gains=None):
    """Every S row a layer of the synthesis reads, cut to the layer's width, as contiguous [N, width] tensors from
    ONE gather (index_select) -- the per-layer views styles[:, r, :width] would each cost a copy kernel (the layers
    take contiguous style rows).  Returns ({row: tensor}, block): rows in `full` keep all columns (the trainable
    rows: delta is added before the cut); rows past until_k are not gathered.  The rows of `lead` (all of them
    gathered, in `full`) come first, in that order, and `block` is them as one [len(lead), N, C] tensor (else None).
    Rows in `gains` ({row: float}, not in `lead`) come next and are returned times their gain, all in one multiply
    (the ToRGB layers' weight_gain: per layer, one small kernel each)."""
    n = styles.shape[0]
    specs = []
    row = 0
    for k, res in enumerate(G.synthesis.block_resolutions):
        width = 2 if res == 4 else 3
        if k <= until_k:
            sh = temp_shapes[k]
            widths = (sh[0], sh[2]) if res == 4 else tuple(sh)
            specs += [(row + j, styles.shape[2] if row + j in full else widths[j]) for j in range(width)]
        row += width
    rows = {r for r, _ in specs}
    lead = tuple(lead) if lead and all(r in rows and r in full for r in lead) else ()
    gains = {r: g for r, g in (gains or {}).items() if r in rows and r not in lead}
    scaled = [sp for sp in specs if sp[0] in gains]
    specs = ([sp for r in lead for sp in specs if sp[0] == r] + scaled +
             [sp for sp in specs if sp[0] not in lead and sp[0] not in gains])
    styles = styles.contiguous()
    key = (n, styles.shape[1], styles.shape[2], tuple(specs), styles.device, tuple(sorted(gains.items())))
    cached = _GATHER_IDX.get(key)
    if cached is None:
        nr, c = styles.shape[1], styles.shape[2]
        base = torch.arange(n).view(n, 1) * (nr * c)
        idx = torch.cat([(base + r * c + torch.arange(w).view(1, w)).reshape(-1) for r, w in specs]).to(styles.device)
        # float32 gains, element by element: the product is the layer's own `styles * weight_gain`, bit for bit
        gvec = torch.cat([torch.full((n * w,), gains[r], dtype=torch.float32) for r, w in scaled]).to(styles.device) \
            if scaled else None
        cached = _GATHER_IDX[key] = (idx, gvec)
    idx, gvec = cached
    flat = styles.reshape(-1).index_select(0, idx)
    if gvec is not None:  # in place: `flat` is this call's own gather
        s0 = len(lead) * n * styles.shape[2]
        flat[s0:s0 + gvec.numel()].mul_(gvec)
    out, off = {}, 0
    for r, w in specs:
        out[r] = flat[off:off + n * w].view(n, w)
        off += n * w
    block = flat[:len(lead) * n * styles.shape[2]].view(len(lead), n, styles.shape[2]) if lead else None
    return out, block


def generate_image_rows(G, until_k, styles, temp_shapes, noise_mode="const", delta=None,
                        trainable=S_TRAINABLE_SPACE_CHANNELS):
    """generate_image(G, until_k, styles + direction) where the direction lives only on `trainable` rows.

    Same arithmetic as block_forward/generate_image, but each S row is passed to its layer as its own
    tensor: only the rows that carry `delta` ([N or 1, len(trainable), 512]) require grad, so the
    backward skips every style gradient find_direction does not use and stops below the first
    trainable layer.  styles2[:, r] = styles[:, r] + delta[:, j] for r = trainable[j] (find_direction.py:307-308).
    The trainable rows are gathered as one [T, N, 512] block and delta is added to it in one op: per row
    (a select, an add and its batch sum), the backward cost ~5 small kernels a row on the critical path.
    """
    x = img = None
    trainable = list(trainable)
    # the ToRGB rows are handed over pre-scaled (affine(w) * weight_gain with affine = Identity, applied in the
    # gather) only when get_temp_shapes has replaced every ToRGB affine; with an intact affine the layer applies
    # affine and gain itself, as generate_image does
    rgb_prescaled = all(isinstance(getattr(G.synthesis, f"b{res}").torgb.affine, torch.nn.Identity)
                        for res in G.synthesis.block_resolutions)
    gains = {}
    row = 0
    for k, res in enumerate(G.synthesis.block_resolutions):
        row += 2 if res == 4 else 3
        if rgb_prescaled:
            gains[row - 1] = getattr(G.synthesis, f"b{res}").torgb.weight_gain
    row = 0
    gathered, block = _gather_rows(G, until_k, styles, temp_shapes, full=set(trainable) if delta is not None else (),
                                   lead=trainable if delta is not None else (), gains=gains)
    edited = None
    if block is not None:
        edited = (block + delta.reshape(-1, len(trainable), block.shape[2]).transpose(0, 1)).unbind(0)
    for k, res in enumerate(G.synthesis.block_resolutions):
        if k > until_k:
            continue
        block_k = getattr(G.synthesis, f"b{res}")
        width = 2 if res == 4 else 3
        rows = []
        for j in range(width):
            r = row + j
            w = gathered[r]
            if delta is not None and r in trainable:
                w = edited[trainable.index(r)] if edited is not None else w + delta[:, trainable.index(r)]
            rows.append(w)
        shapes = temp_shapes[k]
        if block_k.in_channels == 0:
            x = block_k.const.to(torch.float32).unsqueeze(0).repeat([styles.shape[0], 1, 1, 1])
            w1 = rows[0][..., :shapes[0]]
        else:
            x = block_k.conv0(x, rows[0][..., :shapes[0]], noise_mode=noise_mode)
            w1 = rows[1][..., :shapes[1]]
        if img is not None:
            img = upfirdn2d.upsample2d(img, block_k.resample_filter)
        # conv1 + ToRGB as one Function: the backward sums the block output's two gradients (ToRGB and the next
        # block's conv0) inside conv1's epilogue backward
        x, y = block_k.conv1_torgb(x, w1, rows[-1][..., :shapes[2]], noise_mode=noise_mode,
                                   rgb_scaled=rgb_prescaled and ((row + width - 1) not in trainable or delta is None))
        img = img.add_(y) if img is not None else y
        row += width
    return img


def get_temp_shapes(G):
    shapes = []
    for res in G.synthesis.block_resolutions:
        block = getattr(G.synthesis, f"b{res}")
        if res == 4:
            width = block.conv1.affine.weight.shape[0]
            shapes.append((width, width, block.torgb.affine.weight.shape[0]))
            block.conv1.affine = torch.nn.Identity()
        else:
            shapes.append((block.conv0.affine.weight.shape[0], block.conv1.affine.weight.shape[0],
                           block.torgb.affine.weight.shape[0]))
            block.conv0.affine = torch.nn.Identity()
            block.conv1.affine = torch.nn.Identity()
        block.torgb.affine = torch.nn.Identity()
    return shapes


def split_ws(G, ws):
    out = []
    idx = 0
    ws = ws.to(torch.float32)
    for res in G.synthesis.block_resolutions:
        block = getattr(G.synthesis, f"b{res}")
        out.append(ws.narrow(1, idx, block.num_conv + block.num_torgb))
        idx += block.num_conv
    return out


@torch.no_grad()
def get_styles(G, ws, block_ws=None, device=None):
    """W [n, num_ws, 512] -> packed S [n, 26, 512] (zero padded) + temp shapes; mutates G (affines -> Identity)."""
    if block_ws is None:
        block_ws = split_ws(G, ws)
    styles = torch.zeros(ws.size(0), N_STYLE_CHANNELS, 512, device=device or ws.device)
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


def get_mean_std(device):
    mean = torch.as_tensor((0.48145466, 0.4578275, 0.40821073), dtype=torch.float, device=device).view(-1, 1, 1)
    std = torch.as_tensor((0.26862954, 0.26130258, 0.27577711), dtype=torch.float, device=device).view(-1, 1, 1)
    return mean, std
