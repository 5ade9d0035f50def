"""Deterministic synthetic weights and inputs (no checkpoints exist offline).

Every tensor of a state_dict is drawn from its own ``torch.Generator`` seeded by
``(seed, crc32(key))``, so the same key gets the same values no matter which implementation
(product, oracle, reference, HF stand-in) owns the module -- that is what lets the parity tests
load identical weights into independently written models.

Generator weights follow SURVEY.md section 8(d): config-f (channel_base 32768, channel_max 512,
filter [1,3,3,1], skip architecture, conv_clamp 256); conv/affine weights ~N(0,1) (the layers apply
their own equalised-lr gains), biases and noise strengths ~N(0, 0.1), noise_const / const ~N(0,1),
affine biases 1 + N(0, 0.1).  S codes default to N(1, 0.5) ([n, 26, 512], seed 0).
"""
import math
import zlib

import numpy as np
import torch

N_STYLE_CHANNELS = 26


def _gen(seed, key):
    g = torch.Generator()
    g.manual_seed((int(seed) * 1000003 + zlib.crc32(key.encode())) % (2 ** 63 - 1))
    return g


def _normal(shape, seed, key, std=1.0, mean=0.0):
    return torch.randn(tuple(shape), generator=_gen(seed, key)) * std + mean


# ----------------------------------------------------------------------------- generator


def generator_config(resolution=1024, channel_base=None, channel_max=512, conv_clamp=256, w_dim=512, z_dim=512):
    if channel_base is None:
        channel_base = 32768 if resolution >= 512 else 16384   # config-f vs paper256
    return dict(z_dim=z_dim, c_dim=0, w_dim=w_dim, img_resolution=resolution, img_channels=3,
                channel_base=channel_base, channel_max=channel_max, conv_clamp=conv_clamp)


def generator_layer_shapes(cfg):
    """{state_dict key: shape} for the generator of ``cfg`` (legacy.py:172-203 naming)."""
    res_log2 = int(math.log2(cfg["img_resolution"]))
    resolutions = [2 ** i for i in range(2, res_log2 + 1)]
    ch = {r: min(cfg["channel_base"] // r, cfg["channel_max"]) for r in resolutions}
    w = cfg["w_dim"]
    shapes = {}
    for r in resolutions:
        p = f"synthesis.b{r}."
        layers = []
        if r == 4:
            shapes[p + "const"] = (ch[4], 4, 4)
        else:
            layers.append(("conv0", ch[r // 2], ch[r], 3))
        layers.append(("conv1", ch[r], ch[r], 3))
        for name, cin, cout, k in layers:
            q = p + name + "."
            shapes[q + "weight"] = (cout, cin, k, k)
            shapes[q + "bias"] = (cout,)
            shapes[q + "noise_const"] = (r, r)
            shapes[q + "noise_strength"] = ()
            shapes[q + "affine.weight"] = (cin, w)
            shapes[q + "affine.bias"] = (cin,)
        q = p + "torgb."
        shapes[q + "weight"] = (cfg["img_channels"], ch[r], 1, 1)
        shapes[q + "bias"] = (cfg["img_channels"],)
        shapes[q + "affine.weight"] = (ch[r], w)
        shapes[q + "affine.bias"] = (ch[r],)
    feats = [cfg["z_dim"]] + [w] * 8
    for i in range(8):
        shapes[f"mapping.fc{i}.weight"] = (feats[i + 1], feats[i])
        shapes[f"mapping.fc{i}.bias"] = (feats[i + 1],)
    shapes["mapping.w_avg"] = (w,)
    return shapes


def generator_state_dict(cfg, seed=0, lr_multiplier=0.01):
    sd = {}
    for key, shape in generator_layer_shapes(cfg).items():
        leaf = key.rsplit(".", 1)[-1]
        if key.startswith("mapping."):
            if leaf == "weight":
                t = _normal(shape, seed, key) / lr_multiplier
            elif leaf == "bias":
                t = _normal(shape, seed, key, 0.1)
            else:  # w_avg
                t = _normal(shape, seed, key, 0.5)
        elif key.endswith("affine.bias"):
            t = _normal(shape, seed, key, 0.1, 1.0)
        elif leaf in ("bias", "noise_strength"):
            t = _normal(shape, seed, key, 0.1)
        else:  # weight, affine.weight, noise_const, const
            t = _normal(shape, seed, key)
        sd[key] = t.float()
    return sd


def synthetic_styles(n, seed=0, mean=1.0, std=0.5):
    g = torch.Generator()
    g.manual_seed(seed)
    return torch.randn(n, N_STYLE_CHANNELS, 512, generator=g) * std + mean


def seed_latents(seeds, z_dim=512):
    """z for each seed exactly as generate_w.py:48 draws it (float64 -> float32)."""
    return torch.from_numpy(np.concatenate([np.random.RandomState(s).randn(1, z_dim) for s in seeds])).float()


# ----------------------------------------------------------------------------- loss nets


def seeded_state_dict(module, seed=0):
    """Fill any module's parameters/buffers deterministically by key (loss networks).

    conv / linear weights ~ N(0, 1/fan_in); norm weights 1 + N(0, 0.05), biases N(0, 0.02); BN running
    stats mean N(0, 0.05), var 1 + |N(0, 0.1)|; PReLU slopes 0.25; embeddings / projections N(0, d^-1/2).
    """
    out = {}
    for key, ref in module.state_dict().items():
        shape = tuple(ref.shape)
        leaf = key.rsplit(".", 1)[-1]
        if ref.dtype not in (torch.float32, torch.float64, torch.float16):
            out[key] = ref.clone()
            continue
        if leaf == "running_mean":
            t = _normal(shape, seed, key, 0.05)
        elif leaf == "running_var":
            t = 1.0 + _normal(shape, seed, key, 0.1).abs()
        elif "prelu" in key.lower() or _is_prelu(module, key):
            t = torch.full(shape, 0.25)
        elif len(shape) >= 2 and leaf in ("weight", "in_proj_weight"):
            fan_in = int(np.prod(shape[1:]))
            t = _normal(shape, seed, key, 1.0 / math.sqrt(fan_in))
        elif len(shape) == 1 and leaf == "weight":
            t = _normal(shape, seed, key, 0.05, 1.0)
        elif leaf in ("bias", "in_proj_bias"):
            t = _normal(shape, seed, key, 0.02)
        else:  # class_embedding, positional_embedding, proj, ...
            d = shape[0] if len(shape) == 1 else shape[-2] if leaf == "proj" else shape[-1]
            t = _normal(shape, seed, key, 1.0 / math.sqrt(d))
        out[key] = t.to(ref.dtype)
    return out


def _is_prelu(module, key):
    mod = module
    for part in key.split(".")[:-1]:
        mod = getattr(mod, part, None)
        if mod is None:
            return False
    return isinstance(mod, torch.nn.PReLU)


def text_direction(text_prompt, negative_text_prompt, dim=512, seed=0):
    """Seeded stand-in for norm(E_T(pos) - E_T(neg)) when no CLIP text weights exist (clip_loss.py:15-18)."""
    key = f"{text_prompt}\x00{negative_text_prompt}"
    t = _normal((1, dim), seed, "text:" + key)
    return t / t.norm(dim=1, keepdim=True)


def text_embeddings(strings, dim=512, seed=0):
    """Seeded stand-in for E_T(tokenize(s)) per string (un-normalised, [len(strings), dim]) when no CLIP text
    weights exist: the StyleGAN-NADA losses encode 27 templated prompts per class (clip_loss_nada.py:126-136)."""
    return torch.stack([_normal((dim,), seed, "textemb:" + s) for s in strings])
