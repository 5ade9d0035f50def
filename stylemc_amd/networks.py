"""StyleGAN2-ADA generator modules on gfx950 kernels (drop-in for [upstream] training/networks.py).

The reference loads these classes from the network pickle (legacy.py:169, persistence.py:216-227);
``utils.block_forward`` (utils.py:13-53) and ``get_temp_shapes`` (utils.py:100-120) read the attributes
kept here: ``affine`` (replaceable by Identity; ``.weight.shape[0]`` = style width), ``weight``, ``bias``,
``noise_const``, ``noise_strength``, ``up``, ``resolution``, ``conv_clamp``, ``activation``,
``resample_filter``, ``weight_gain``, and per block ``num_conv``, ``num_torgb``, ``w_dim``, ``use_fp16``,
``channels_last``, ``in_channels``, ``const``, ``conv0``, ``conv1``, ``torgb``, ``architecture``,
``resolution``, ``img_channels``, ``is_last``.  Parameter names follow the pickle's state_dict
(legacy.py:172-203) so converted weights load unchanged.

Compute: every SynthesisLayer / ToRGBLayer runs the HIP modconv kernels (stylemc_amd.modconv); the
generator is treated as frozen (no gradients w.r.t. its parameters, only w.r.t. activations and
styles -- which is all find_direction needs).  All blocks compute in fp32 (``use_fp16`` is recorded
for compatibility, never used to lower precision).
"""
import math

import numpy as np
import torch

from . import modconv
from .torch_utils.ops import bias_act as _bias_act
from .torch_utils.ops import upfirdn2d as _upfirdn2d


def normalize_2nd_moment(x, dim=1, eps=1e-8):
    return x * (x.square().mean(dim=dim, keepdim=True) + eps).rsqrt()


class FullyConnectedLayer(torch.nn.Module):
    def __init__(self, in_features, out_features, bias=True, activation="linear", lr_multiplier=1.0, bias_init=0.0):
        super().__init__()
        self.activation = activation
        self.weight = torch.nn.Parameter(torch.randn(out_features, in_features) / lr_multiplier)
        self.bias = torch.nn.Parameter(torch.full([out_features], float(bias_init))) if bias else None
        self.weight_gain = lr_multiplier / math.sqrt(in_features)
        self.bias_gain = lr_multiplier

    def forward(self, x):
        w = self.weight.to(x.dtype) * self.weight_gain
        b = self.bias
        if b is not None:
            b = b.to(x.dtype)
            if self.bias_gain != 1:
                b = b * self.bias_gain
        if self.activation == "linear" and b is not None:
            return torch.addmm(b.unsqueeze(0), x, w.t())
        return _bias_act.bias_act(x.matmul(w.t()), b, act=self.activation)


class _SpecCache:
    """Rebuild the packed-weight spec only when the layer's parameters change."""

    def __init__(self):
        self.key = None
        self.spec = None

    def get(self, key, build):
        if key != self.key:
            self.spec = build()
            self.key = key
        return self.spec


def _version_key(*tensors):
    return tuple((t.data_ptr(), t._version, str(t.device)) if t is not None else None for t in tensors)


class SynthesisLayer(torch.nn.Module):
    def __init__(self, in_channels, out_channels, w_dim, resolution, kernel_size=3, up=1, use_noise=True,
                 activation="lrelu", resample_filter=(1, 3, 3, 1), conv_clamp=None, channels_last=False):
        super().__init__()
        self.resolution = resolution
        self.up = up
        self.use_noise = use_noise
        self.activation = activation
        self.conv_clamp = conv_clamp
        self.register_buffer("resample_filter", _upfirdn2d.setup_filter(list(resample_filter)))
        self.padding = kernel_size // 2
        self.act_gain = _bias_act.activation_funcs[activation].def_gain
        self.affine = FullyConnectedLayer(w_dim, in_channels, bias_init=1)
        self.weight = torch.nn.Parameter(torch.randn(out_channels, in_channels, kernel_size, kernel_size))
        if use_noise:
            self.register_buffer("noise_const", torch.randn(resolution, resolution))
            self.noise_strength = torch.nn.Parameter(torch.zeros([]))
        self.bias = torch.nn.Parameter(torch.zeros(out_channels))
        self._spec = _SpecCache()

    def spec(self):
        alpha = _bias_act.activation_funcs[self.activation].def_alpha
        return self._spec.get(_version_key(self.weight, self.bias, self.resample_filter),
                              lambda: modconv.LayerSpec(self.weight, self.bias, self.up, self.resample_filter,
                                                        demodulate=True, act=self.activation, alpha=alpha,
                                                        resolution=self.resolution))

    def fn_args(self, x, w, noise_mode="random", gain=1):
        """The ModConvFn argument tuple of forward(x, w, noise_mode, gain=gain)."""
        assert noise_mode in ("random", "const", "none")
        in_res = self.resolution // self.up
        assert x.shape[1:] == (self.weight.shape[1], in_res, in_res), (tuple(x.shape), self.weight.shape)
        styles = self.affine(w)
        noise = strength = None
        if self.use_noise and noise_mode == "random":
            noise = torch.randn([x.shape[0], 1, self.resolution, self.resolution], device=x.device)
        if self.use_noise and noise_mode == "const":
            noise = self.noise_const
        if noise is not None:
            strength = self.noise_strength.detach()
        act_gain = float(self.act_gain * gain)
        act_clamp = float(self.conv_clamp * gain) if self.conv_clamp is not None else -1.0
        return x.float(), styles.float(), self.spec(), noise, strength, act_gain, act_clamp

    def forward(self, x, w, noise_mode="random", fused_modconv=True, gain=1):
        return modconv.ModConvFn.apply(*self.fn_args(x, w, noise_mode, gain))


class ToRGBLayer(torch.nn.Module):
    def __init__(self, in_channels, out_channels, w_dim, kernel_size=1, conv_clamp=None, channels_last=False):
        super().__init__()
        assert kernel_size == 1
        self.conv_clamp = conv_clamp
        self.affine = FullyConnectedLayer(w_dim, in_channels, bias_init=1)
        self.weight = torch.nn.Parameter(torch.randn(out_channels, in_channels, kernel_size, kernel_size))
        self.bias = torch.nn.Parameter(torch.zeros(out_channels))
        self.weight_gain = 1 / math.sqrt(in_channels * kernel_size * kernel_size)
        self._w2d = _SpecCache()

    def fn_args(self, x, w, scaled=False):
        """The ToRGBFn argument tuple of forward(x, w); scaled: w is already affine(w) * weight_gain."""
        styles = w if scaled else self.affine(w) * self.weight_gain
        w2d = self._w2d.get(_version_key(self.weight), self._pack_w2d)
        clamp = float(self.conv_clamp) if self.conv_clamp is not None else -1.0
        return x.float(), styles.float(), w2d, self.bias.detach().float().contiguous(), clamp

    def _pack_w2d(self):
        w2d = self.weight.detach()[:, :, 0, 0].float().contiguous()
        if w2d.is_cuda:  # built on whichever stream first reaches the layer; other streams read it right after
            torch.cuda.current_stream(w2d.device).synchronize()
        return w2d

    def forward(self, x, w, fused_modconv=True):
        return modconv.ToRGBFn.apply(*self.fn_args(x, w))


class SynthesisBlock(torch.nn.Module):
    def __init__(self, in_channels, out_channels, w_dim, resolution, img_channels, is_last, architecture="skip",
                 resample_filter=(1, 3, 3, 1), conv_clamp=None, use_fp16=False, fp16_channels_last=False,
                 **layer_kwargs):
        super().__init__()
        if architecture != "skip":
            raise NotImplementedError("only the 'skip' architecture (all FFHQ configs) is implemented")
        self.in_channels = in_channels
        self.w_dim = w_dim
        self.resolution = resolution
        self.img_channels = img_channels
        self.is_last = is_last
        self.architecture = architecture
        self.use_fp16 = use_fp16
        self.channels_last = use_fp16 and fp16_channels_last
        self.register_buffer("resample_filter", _upfirdn2d.setup_filter(list(resample_filter)))
        self.num_conv = 0
        self.num_torgb = 0
        if in_channels == 0:
            self.const = torch.nn.Parameter(torch.randn(out_channels, resolution, resolution))
        else:
            self.conv0 = SynthesisLayer(in_channels, out_channels, w_dim, resolution, up=2,
                                        resample_filter=resample_filter, conv_clamp=conv_clamp, **layer_kwargs)
            self.num_conv += 1
        self.conv1 = SynthesisLayer(out_channels, out_channels, w_dim, resolution, conv_clamp=conv_clamp,
                                    **layer_kwargs)
        self.num_conv += 1
        self.torgb = ToRGBLayer(out_channels, img_channels, w_dim, conv_clamp=conv_clamp)
        self.num_torgb += 1

    def conv1_torgb(self, x, w1, w_rgb, noise_mode="random", rgb_scaled=False):
        """conv1(x, w1) and the ToRGB of its output as one autograd Function (modconv.ModConvToRGBFn, whose
        backward fuses the two gradients of the block output): returns (x, rgb) = (conv1 output, ToRGB output).
        rgb_scaled: w_rgb is already the ToRGB styles (affine(w_rgb) * weight_gain, see utils._gather_rows)."""
        return modconv.ModConvToRGBFn.apply(*self.conv1.fn_args(x, w1, noise_mode),
                                            *self.torgb.fn_args(x, w_rgb, scaled=rgb_scaled)[1:])

    def forward(self, x, img, ws, force_fp32=False, fused_modconv=None, **layer_kwargs):
        rows = iter(ws.unbind(dim=1))
        if self.in_channels == 0:
            x = self.const.float().unsqueeze(0).repeat([ws.shape[0], 1, 1, 1])
        else:
            x = self.conv0(x, next(rows), **layer_kwargs)
        x = self.conv1(x, next(rows), **layer_kwargs)
        if img is not None:
            img = _upfirdn2d.upsample2d(img, self.resample_filter)
        y = self.torgb(x, next(rows))
        img = img.add_(y) if img is not None else y
        return x, img


class SynthesisNetwork(torch.nn.Module):
    def __init__(self, w_dim, img_resolution, img_channels, channel_base=32768, channel_max=512, num_fp16_res=0,
                 **block_kwargs):
        super().__init__()
        assert img_resolution >= 4 and img_resolution & (img_resolution - 1) == 0
        self.w_dim = w_dim
        self.img_resolution = img_resolution
        self.img_resolution_log2 = int(np.log2(img_resolution))
        self.img_channels = img_channels
        self.block_resolutions = [2 ** i for i in range(2, self.img_resolution_log2 + 1)]
        ch = {r: min(channel_base // r, channel_max) for r in self.block_resolutions}
        fp16_resolution = max(2 ** (self.img_resolution_log2 + 1 - num_fp16_res), 8)
        self.num_ws = 0
        for res in self.block_resolutions:
            block = SynthesisBlock(ch[res // 2] if res > 4 else 0, ch[res], w_dim=w_dim, resolution=res,
                                   img_channels=img_channels, is_last=(res == img_resolution),
                                   use_fp16=(res >= fp16_resolution), **block_kwargs)
            self.num_ws += block.num_conv
            if res == img_resolution:
                self.num_ws += block.num_torgb
            setattr(self, f"b{res}", block)

    def forward(self, ws, **block_kwargs):
        x = img = None
        w_idx = 0
        for res in self.block_resolutions:
            block = getattr(self, f"b{res}")
            cur = ws.narrow(1, w_idx, block.num_conv + block.num_torgb)
            w_idx += block.num_conv
            x, img = block(x, img, cur, **block_kwargs)
        return img


class MappingNetwork(torch.nn.Module):
    """z -> W (8 FC lrelu layers, lr_multiplier 0.01, normalize_2nd_moment, truncation vs w_avg)."""

    def __init__(self, z_dim, c_dim, w_dim, num_ws, num_layers=8, lr_multiplier=0.01, w_avg_beta=0.995):
        super().__init__()
        if c_dim != 0:
            raise NotImplementedError("conditional mapping networks are not supported")
        self.z_dim, self.c_dim, self.w_dim, self.num_ws, self.num_layers = z_dim, c_dim, w_dim, num_ws, num_layers
        feats = [z_dim] + [w_dim] * num_layers
        for i in range(num_layers):
            setattr(self, f"fc{i}", FullyConnectedLayer(feats[i], feats[i + 1], activation="lrelu",
                                                        lr_multiplier=lr_multiplier))
        self.register_buffer("w_avg", torch.zeros(w_dim))

    def forward(self, z, c=None, truncation_psi=1, truncation_cutoff=None):
        x = normalize_2nd_moment(z.to(torch.float32))
        for i in range(self.num_layers):
            x = getattr(self, f"fc{i}")(x)
        x = x.unsqueeze(1).repeat([1, self.num_ws, 1])
        if truncation_psi != 1:
            if truncation_cutoff is None:
                x = self.w_avg.lerp(x, truncation_psi)
            else:
                x[:, :truncation_cutoff] = self.w_avg.lerp(x[:, :truncation_cutoff], truncation_psi)
        return x


class Generator(torch.nn.Module):
    def __init__(self, z_dim, c_dim, w_dim, img_resolution, img_channels, mapping_kwargs=None, **synthesis_kwargs):
        super().__init__()
        self.z_dim, self.c_dim, self.w_dim = z_dim, c_dim, w_dim
        self.img_resolution, self.img_channels = img_resolution, img_channels
        self.synthesis = SynthesisNetwork(w_dim=w_dim, img_resolution=img_resolution, img_channels=img_channels,
                                          **synthesis_kwargs)
        self.num_ws = self.synthesis.num_ws
        self.mapping = MappingNetwork(z_dim=z_dim, c_dim=c_dim, w_dim=w_dim, num_ws=self.num_ws,
                                      **(mapping_kwargs or {}))

    def forward(self, z, c=None, truncation_psi=1, truncation_cutoff=None, **synthesis_kwargs):
        ws = self.mapping(z, c, truncation_psi=truncation_psi, truncation_cutoff=truncation_cutoff)
        return self.synthesis(ws, **synthesis_kwargs)


def infer_generator_config(state_dict, conv_clamp=256):
    """Generator config from a G_ema state_dict's shapes (legacy.py:172-203 names): img_resolution from the
    highest ``synthesis.b{R}`` block, per-block widths -> channel_base / channel_max, z_dim / w_dim / mapping
    depth from the mapping and affine FCs.  conv_clamp is not stored in a state_dict (the stylegan2-ada
    training configs use 256; converted TF-era networks use None)."""
    import re
    res = sorted({int(m.group(1)) for k in state_dict for m in [re.match(r"synthesis\.b(\d+)\.", k)] if m})
    if not res or res[0] != 4:
        raise KeyError("not a StyleGAN2 generator state_dict (no synthesis.b4.* keys)")
    R = res[-1]
    ch = {r: int(state_dict[f"synthesis.b{r}.conv1.weight"].shape[0]) for r in res}
    channel_max = max(ch.values())
    below = [ch[r] * r for r in res if ch[r] < channel_max]
    channel_base = min(below) if below else channel_max * R
    if any(min(channel_base // r, channel_max) != ch[r] for r in res):
        raise ValueError(f"block widths {ch} do not follow min(channel_base / r, channel_max)")
    w_dim = int(state_dict["synthesis.b4.conv1.affine.weight"].shape[1])
    n_map = len({k.split(".")[1] for k in state_dict if re.match(r"mapping\.fc\d+\.weight$", k)})
    z_dim = int(state_dict["mapping.fc0.weight"].shape[1]) if n_map else 512
    return dict(z_dim=z_dim, c_dim=0, w_dim=w_dim, img_resolution=R,
                img_channels=int(state_dict[f"synthesis.b{R}.torgb.weight"].shape[0]), channel_base=channel_base,
                channel_max=channel_max, conv_clamp=conv_clamp, mapping_layers=n_map or 8)


def build_generator(cfg, state_dict=None, device="cuda"):
    """Generator from a ``synthetic.generator_config`` dict (+ optional state_dict), frozen, on ``device``."""
    G = Generator(cfg["z_dim"], cfg["c_dim"], cfg["w_dim"], cfg["img_resolution"], cfg["img_channels"],
                  mapping_kwargs=dict(num_layers=cfg.get("mapping_layers", 8)), channel_base=cfg["channel_base"],
                  channel_max=cfg["channel_max"], conv_clamp=cfg["conv_clamp"])
    if state_dict is not None:
        res = G.load_state_dict(state_dict, strict=False)
        bad = [k for k in res.missing_keys if not k.endswith("resample_filter")]
        if bad or res.unexpected_keys:
            raise KeyError(f"state_dict mismatch: missing={bad} unexpected={res.unexpected_keys}")
    return G.eval().requires_grad_(False).to(device)
