"""CPU restatement of the StyleGAN2-ADA generator layers (TEST ORACLE ONLY).

The reference imports these from NVlabs stylegan2-ada-pytorch ``training/networks.py``
(``legacy.py:169``), which is NOT vendored in /root/reference -- the classes normally arrive as
source text inside the network pickle (``torch_utils/persistence.py:118-126,216-227``).  This module
restates the published upstream semantics; every attribute read by the reference's
``utils.block_forward`` (utils.py:13-53) / ``get_temp_shapes`` (utils.py:100-120) is provided.

Parameter names follow the pickle's state_dict contract (legacy.py:172-203):
``synthesis.b{r}.conv{0,1}.{weight,bias,noise_const,noise_strength,affine.weight,affine.bias}``,
``synthesis.b{r}.torgb.*``, ``synthesis.b4.const``, ``mapping.fc{i}.*``, ``mapping.w_avg``.
"""
import math

import numpy as np
import torch

from . import ops


def normalize_2nd_moment(x, dim=1, eps=1e-8):
    return x * (x.square().mean(dim=dim, keepdim=True) + eps).rsqrt()


class FullyConnectedLayer(torch.nn.Module):
    """Equalized-lr linear layer ([upstream] FullyConnectedLayer)."""

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
        return ops.bias_act(x.matmul(w.t()), b, act=self.activation)


def modulated_conv2d(x, weight, styles, noise=None, up=1, down=1, padding=0, resample_filter=None,
                     demodulate=True, flip_weight=True, fused_modconv=True):
    """[upstream] modulated_conv2d: w_n = W * s_n; d_n = rsqrt(sum w_n^2 + 1e-8); conv; + noise."""
    n = x.shape[0]
    oc, ic, kh, kw = weight.shape
    assert styles.shape == (n, ic)
    if x.dtype == torch.float16 and demodulate:
        weight = weight * (1 / np.sqrt(ic * kh * kw) / weight.norm(float("inf"), dim=[1, 2, 3], keepdim=True))
        styles = styles / styles.norm(float("inf"), dim=1, keepdim=True)
    w = dcoefs = None
    if demodulate or fused_modconv:
        w = weight.unsqueeze(0) * styles.reshape(n, 1, -1, 1, 1)          # [N, O, I, k, k]
    if demodulate:
        dcoefs = (w.square().sum(dim=[2, 3, 4]) + 1e-8).rsqrt()           # [N, O]
    if demodulate and fused_modconv:
        w = w * dcoefs.reshape(n, -1, 1, 1, 1)
    if not fused_modconv:
        x = x * styles.to(x.dtype).reshape(n, -1, 1, 1)
        x = ops.conv2d_resample(x, weight.to(x.dtype), f=resample_filter, up=up, down=down,
                                padding=padding, flip_weight=flip_weight)
        if demodulate and noise is not None:
            x = ops.fma(x, dcoefs.to(x.dtype).reshape(n, -1, 1, 1), noise.to(x.dtype))
        elif demodulate:
            x = x * dcoefs.to(x.dtype).reshape(n, -1, 1, 1)
        elif noise is not None:
            x = x.add_(noise.to(x.dtype))
        return x
    # Fused: one grouped convolution with per-sample weights.
    x = x.reshape(1, -1, *x.shape[2:])
    w = w.reshape(-1, ic, kh, kw)
    x = ops.conv2d_resample(x, w.to(x.dtype), f=resample_filter, up=up, down=down, padding=padding,
                            groups=n, flip_weight=flip_weight)
    x = x.reshape(n, -1, *x.shape[2:])
    if noise is not None:
        x = x.add_(noise)
    return x


class SynthesisLayer(torch.nn.Module):
    def __init__(self, in_channels, out_channels, w_dim, resolution, kernel_size=3, up=1, use_noise=True,
                 activation="lrelu", resample_filter=(1, 3, 3, 1), conv_clamp=None, channels_last=False):
        super().__init__()
        self.resolution = resolution
        self.up = up
        self.use_noise = use_noise
        self.activation = activation
        self.conv_clamp = conv_clamp
        self.register_buffer("resample_filter", ops.setup_filter(list(resample_filter)))
        self.padding = kernel_size // 2
        self.act_gain = ops.act_defaults(activation)[1]
        self.affine = FullyConnectedLayer(w_dim, in_channels, bias_init=1)
        self.weight = torch.nn.Parameter(torch.randn(out_channels, in_channels, kernel_size, kernel_size))
        if use_noise:
            self.register_buffer("noise_const", torch.randn(resolution, resolution))
            self.noise_strength = torch.nn.Parameter(torch.zeros([]))
        self.bias = torch.nn.Parameter(torch.zeros(out_channels))

    def forward(self, x, w, noise_mode="random", fused_modconv=True, gain=1):
        assert noise_mode in ("random", "const", "none")
        styles = self.affine(w)
        noise = None
        if self.use_noise and noise_mode == "random":
            noise = torch.randn(x.shape[0], 1, self.resolution, self.resolution, device=x.device) * self.noise_strength
        if self.use_noise and noise_mode == "const":
            noise = self.noise_const * self.noise_strength
        x = modulated_conv2d(x, self.weight, styles, noise=noise, up=self.up, padding=self.padding,
                             resample_filter=self.resample_filter, flip_weight=(self.up == 1),
                             fused_modconv=fused_modconv)
        act_gain = self.act_gain * gain
        act_clamp = self.conv_clamp * gain if self.conv_clamp is not None else None
        return ops.bias_act(x, self.bias.to(x.dtype), act=self.activation, gain=act_gain, clamp=act_clamp)


class ToRGBLayer(torch.nn.Module):
    def __init__(self, in_channels, out_channels, w_dim, kernel_size=1, conv_clamp=None, channels_last=False):
        super().__init__()
        self.conv_clamp = conv_clamp
        self.affine = FullyConnectedLayer(w_dim, in_channels, bias_init=1)
        self.weight = torch.nn.Parameter(torch.randn(out_channels, in_channels, kernel_size, kernel_size))
        self.bias = torch.nn.Parameter(torch.zeros(out_channels))
        self.weight_gain = 1 / math.sqrt(in_channels * kernel_size * kernel_size)

    def forward(self, x, w, fused_modconv=True):
        styles = self.affine(w) * self.weight_gain
        x = modulated_conv2d(x, self.weight, styles, demodulate=False, fused_modconv=fused_modconv)
        return ops.bias_act(x, self.bias.to(x.dtype), clamp=self.conv_clamp)


class SynthesisBlock(torch.nn.Module):
    def __init__(self, in_channels, out_channels, w_dim, resolution, img_channels, is_last, architecture="skip",
                 resample_filter=(1, 3, 3, 1), conv_clamp=None, use_fp16=False, fp16_channels_last=False,
                 **layer_kwargs):
        super().__init__()
        assert architecture == "skip", "only the skip architecture (FFHQ configs) is restated"
        self.in_channels = in_channels
        self.w_dim = w_dim
        self.resolution = resolution
        self.img_channels = img_channels
        self.is_last = is_last
        self.architecture = architecture
        self.use_fp16 = use_fp16
        self.channels_last = use_fp16 and fp16_channels_last
        self.register_buffer("resample_filter", ops.setup_filter(list(resample_filter)))
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

    def forward(self, x, img, ws, force_fp32=False, fused_modconv=None, **layer_kwargs):
        w_iter = iter(ws.unbind(dim=1))
        if fused_modconv is None:
            fused_modconv = not self.training
        if self.in_channels == 0:
            x = self.const.unsqueeze(0).repeat([ws.shape[0], 1, 1, 1])
        else:
            x = self.conv0(x, next(w_iter), fused_modconv=fused_modconv, **layer_kwargs)
        x = self.conv1(x, next(w_iter), fused_modconv=fused_modconv, **layer_kwargs)
        if img is not None:
            img = ops.upsample2d(img, self.resample_filter)
        y = self.torgb(x, next(w_iter), fused_modconv=fused_modconv).to(torch.float32)
        img = img.add_(y) if img is not None else y
        return x, img


def channels_for(res, channel_base, channel_max):
    return min(channel_base // res, channel_max)


class SynthesisNetwork(torch.nn.Module):
    def __init__(self, w_dim, img_resolution, img_channels, channel_base=32768, channel_max=512, num_fp16_res=0,
                 **block_kwargs):
        super().__init__()
        self.w_dim = w_dim
        self.img_resolution = img_resolution
        self.img_resolution_log2 = int(np.log2(img_resolution))
        self.img_channels = img_channels
        self.block_resolutions = [2 ** i for i in range(2, self.img_resolution_log2 + 1)]
        ch = {r: channels_for(r, channel_base, channel_max) for r in self.block_resolutions}
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
    def __init__(self, z_dim, c_dim, w_dim, num_ws, num_layers=8, lr_multiplier=0.01, w_avg_beta=0.995):
        super().__init__()
        assert c_dim == 0, "unconditional generators only"
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
