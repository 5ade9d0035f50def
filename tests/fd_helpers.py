"""Oracle-backed pieces that let stylemc_amd.find_direction.DirectionFinder run on the CPU in tests
(multi-process gloo coverage) and provide the CPU reference for the GPU parity tests."""
import torch

from oracle import losses as OL
from oracle import networks as ON
from oracle import ops as O
from stylemc_amd import synthetic
from stylemc_amd.utils import S_TRAINABLE_SPACE_CHANNELS


def oracle_generator(res, cbase, clamp=256.0, seed=0):
    cfg = synthetic.generator_config(resolution=res, channel_base=cbase, conv_clamp=clamp)
    sd = synthetic.generator_state_dict(cfg, seed=seed)
    G = torch.nn.Module()
    G.synthesis = ON.SynthesisNetwork(512, res, 3, channel_base=cbase, conv_clamp=clamp)
    r = G.synthesis.load_state_dict({k[10:]: v for k, v in sd.items() if k.startswith("synthesis.")}, strict=False)
    assert not r.unexpected_keys
    return G.eval().requires_grad_(False)


def oracle_rows_synth(G, until_k, styles, temp_shapes, noise_mode="const", delta=None, trainable=S_TRAINABLE_SPACE_CHANNELS):
    """CPU twin of stylemc_amd.utils.generate_image_rows on oracle layers."""
    x = img = None
    row = 0
    for k, res in enumerate(G.synthesis.block_resolutions):
        if k > until_k:
            continue
        block = getattr(G.synthesis, f"b{res}")
        width = 2 if res == 4 else 3
        rows = []
        for j in range(width):
            w = styles[:, row + j]
            if delta is not None and row + j in trainable:
                w = w + delta[:, trainable.index(row + j)]
            rows.append(w)
        sh = temp_shapes[k]
        if block.in_channels == 0:
            x = block.const.unsqueeze(0).repeat([styles.shape[0], 1, 1, 1])
            x = block.conv1(x, rows[0][..., :sh[0]], noise_mode=noise_mode)
        else:
            x = block.conv0(x, rows[0][..., :sh[0]], noise_mode=noise_mode)
            x = block.conv1(x, rows[1][..., :sh[1]], noise_mode=noise_mode)
        if img is not None:
            img = O.upsample2d(img, block.resample_filter)
        y = block.torgb(x, rows[-1][..., :sh[2]])
        img = img + y if img is not None else y
        row += width
    return img


def per_image_synth(G, until_k, styles, temp_shapes, noise_mode="const", delta=None,
                    trainable=S_TRAINABLE_SPACE_CHANNELS):
    """oracle_rows_synth one image at a time: each image's result (and gradient) is then independent of the batch
    it came in -- CPU torch picks conv / matmul algorithms by batch size, so a batched oracle is not."""
    outs = []
    for i in range(styles.shape[0]):
        d = None if delta is None else (delta[i:i + 1] if delta.shape[0] > 1 else delta)
        outs.append(oracle_rows_synth(G, until_k, styles[i:i + 1], temp_shapes, noise_mode, delta=d,
                                      trainable=trainable))
    return torch.cat(outs)


class _PerImage(torch.nn.Module):
    def __init__(self, inner):
        super().__init__()
        self.inner = inner

    def forward(self, x):
        return torch.cat([self.inner(x[i:i + 1]) for i in range(x.shape[0])])


def per_image_module(m):
    """A batch-invariant wrapper: the module applied image by image (see per_image_synth)."""
    return _PerImage(m)


class OracleID(torch.nn.Module):
    def __init__(self, facenet):
        super().__init__()
        self.inner = OL.IDLoss(facenet)

    def target_feats(self, y):
        return self.inner.extract_feats(y).detach()

    def per_sample_with(self, y_hat, f):
        return 1 - (self.inner.extract_feats(y_hat) * f).sum(1)

    def per_sample(self, y_hat, y):
        return self.per_sample_with(y_hat, self.target_feats(y))

    def per_sample_pair(self, y_hat, y):
        n = y_hat.shape[0]
        f = self.inner.extract_feats(torch.cat([y_hat, y.detach()]))
        return 1 - (f[:n] * f[n:].detach()).sum(1)


class OracleCLIP(torch.nn.Module):
    def __init__(self, visual, text):
        super().__init__()
        self.inner = OL.CLIPLoss(visual, text)

    def encode_src(self, src):
        return self.inner.visual(src).detach()

    def per_sample_with(self, e, tgt):
        f = self.inner.visual(tgt) - e
        f = f / f.norm(dim=1, keepdim=True)
        return 1 - torch.nn.functional.cosine_similarity(f, self.inner.text_features)

    def per_sample(self, src, tgt):
        return self.per_sample_with(self.encode_src(src), tgt)

    def per_sample_pair(self, tgt, src):
        n = tgt.shape[0]
        e = self.inner.visual(torch.cat([tgt, src.detach()]))
        f = e[:n] - e[n:].detach()
        f = f / f.norm(dim=1, keepdim=True)
        return 1 - torch.nn.functional.cosine_similarity(f, self.inner.text_features)


class TinyFace(torch.nn.Module):
    """Small stand-in for IR-SE50 (distributed-logic tests only): [N,3,112,112] -> unit [N,32]."""

    def __init__(self):
        super().__init__()
        g = torch.Generator().manual_seed(0)
        self.w1 = torch.nn.Parameter(torch.randn(8, 3, 5, 5, generator=g) * 0.2, requires_grad=False)
        self.w2 = torch.nn.Parameter(torch.randn(32, 8 * 14 * 14, generator=g) * 0.02, requires_grad=False)

    def forward(self, x):
        x = torch.nn.functional.conv2d(x, self.w1, stride=4, padding=2).tanh()
        x = torch.nn.functional.adaptive_avg_pool2d(x, 14).flatten(1) @ self.w2.t()
        return x / x.norm(dim=1, keepdim=True)


def tiny_clip_visual():
    vis = OL.CLIPVisual(input_resolution=224, patch_size=32, width=64, layers=2, heads=2, output_dim=32).eval()
    vis.load_state_dict(synthetic.seeded_state_dict(vis, seed=4))
    return vis.requires_grad_(False)
