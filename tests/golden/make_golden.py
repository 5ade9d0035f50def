"""Generate the golden vectors under tests/golden/ by running the REFERENCE's own code on CPU.

Run here (the container that has /root/reference), never on the GPU box:

    python tests/golden/make_golden.py

What is imported from the reference (read-only, CPU, its pure-torch ``_ref`` paths):
  torch_utils.ops.upfirdn2d / bias_act / conv2d_resample / fma, utils.block_forward /
  utils.generate_image / utils.get_temp_shapes (with a stub ``cv2`` module: cv2 is only used by the
  blending helpers), id_loss.model_irse.Backbone.
The StyleGAN2 layer classes are not in the reference tree; the tiny
generator below evaluates the upstream ``modulated_conv2d`` formula on top of the reference's ops,
so the fixture pins the reference ops + the reference block driver, with the layer formula restated.
CLIP is third-party and absent: its fixture comes from ``transformers.CLIPVisionModelWithProjection``
(ViT-B/32 config, quick_gelu) with the same seeded weights -- an architecture cross-check only.
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, REF)
sys.modules.setdefault("cv2", types.ModuleType("cv2"))

from torch_utils.ops import bias_act as ref_bias_act          # noqa: E402
from torch_utils.ops import conv2d_resample as ref_c2r        # noqa: E402
from torch_utils.ops import fma as ref_fma                     # noqa: E402
from torch_utils.ops import upfirdn2d as ref_upfirdn2d         # noqa: E402
import utils as ref_utils                                      # noqa: E402

from stylemc_amd import synthetic                              # noqa: E402

torch.backends.cudnn.deterministic = True


def save(name, d):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **{k: (v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v))
                                 for k, v in d.items()})
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.1f} KiB, {len(d)} arrays)")


# ---------------------------------------------------------------------------------- ops


def gen_upfirdn2d():
    g = torch.Generator().manual_seed(1)
    f4 = ref_upfirdn2d.setup_filter([1, 3, 3, 1])
    cases = {
        # (x shape, filter, up, down, padding, flip, gain)
        "blur_conv0": ([2, 6, 9, 9], f4, 1, 1, [1, 1, 1, 1], False, 4),          # conv2d_resample.py:139 pattern
        "up2_img": ([2, 3, 8, 8], f4, 2, 1, [2, 1, 2, 1], False, 4),             # upsample2d (utils.py:45)
        "down2_adj": ([2, 3, 16, 16], f4, 1, 2, [1, 2, 1, 2], True, 4),          # adjoint of up2_img
        "blur_adj": ([2, 6, 8, 8], f4, 1, 1, [2, 2, 2, 2], True, 4),             # adjoint of blur_conv0
        "rect_up2_down1": ([1, 2, 5, 7], f4, [2, 1], 1, [2, 1, 0, 3], False, 1),
        "crop_neg_pad": ([1, 2, 12, 10], f4, 1, 2, [-1, 2, 0, -2], False, 2),
        "odd_filter": ([2, 2, 7, 6], ref_upfirdn2d.setup_filter([[1, 2, 1], [2, 4, 3], [0, 1, 1]]), 2, 2,
                       [1, 1, 2, 0], False, 1),
        "sep_filter8": ([1, 3, 11, 13], ref_upfirdn2d.setup_filter([1, 2, 3, 4, 4, 3, 2, 1]), 2, 1,
                        [4, 3, 4, 3], False, 4),
        "up4_down3": ([1, 1, 6, 5], f4, 4, 3, [3, 2, 1, 4], True, 1),
        "single_pixel": ([1, 1, 1, 1], f4, 2, 1, [2, 1, 2, 1], False, 4),
    }
    out = {}
    for name, (shape, f, up, down, pad, flip, gain) in cases.items():
        x = torch.randn(shape, generator=g).requires_grad_(True)
        y = ref_upfirdn2d.upfirdn2d(x, f, up=up, down=down, padding=pad, flip_filter=flip, gain=gain, impl="ref")
        dy = torch.randn(y.shape, generator=g)
        (dx,) = torch.autograd.grad(y, x, dy)
        out.update({f"{name}/x": x, f"{name}/f": f, f"{name}/y": y, f"{name}/dy": dy, f"{name}/dx": dx,
                    f"{name}/up": np.array(up if isinstance(up, list) else [up, up]),
                    f"{name}/down": np.array(down if isinstance(down, list) else [down, down]),
                    f"{name}/pad": np.array(pad), f"{name}/flip": np.array(int(flip)), f"{name}/gain": np.array(gain)})
    # helper wrappers
    x = torch.randn([2, 3, 8, 8], generator=g)
    out["helper/x"] = x
    out["helper/upsample2d"] = ref_upfirdn2d.upsample2d(x, f4, impl="ref")
    out["helper/downsample2d"] = ref_upfirdn2d.downsample2d(x, f4, impl="ref")
    out["helper/filter2d"] = ref_upfirdn2d.filter2d(x, f4, impl="ref")
    out["helper/f4"] = f4
    save("ops_upfirdn2d.npz", out)


def gen_bias_act():
    g = torch.Generator().manual_seed(2)
    out = {}
    acts = ["linear", "relu", "lrelu", "tanh", "sigmoid", "elu", "selu", "softplus", "swish"]
    for act in acts:
        for clamp in (None, 0.7):
            name = f"{act}_c{'none' if clamp is None else clamp}"
            x = (torch.randn([3, 5, 4, 6], generator=g) * 2).requires_grad_(True)
            b = (torch.randn([5], generator=g) * 0.5).requires_grad_(True)
            y = ref_bias_act.bias_act(x, b, act=act, clamp=clamp, impl="ref")
            dy = torch.randn(y.shape, generator=g)
            dx, db = torch.autograd.grad(y, [x, b], dy)
            out.update({f"{name}/x": x, f"{name}/b": b, f"{name}/y": y, f"{name}/dy": dy, f"{name}/dx": dx,
                        f"{name}/db": db})
    # non-default dim / gain / alpha
    x = torch.randn([4, 7], generator=g)
    b = torch.randn([4], generator=g)
    out["dim0/x"], out["dim0/b"] = x, b
    out["dim0/y"] = ref_bias_act.bias_act(x, b, dim=0, act="lrelu", alpha=0.1, gain=3.0, clamp=2.0, impl="ref")
    save("ops_bias_act.npz", out)


def gen_conv2d_resample():
    g = torch.Generator().manual_seed(3)
    f4 = ref_upfirdn2d.setup_filter([1, 3, 3, 1])
    out = {}
    cases = {
        # name: (x shape, w shape, up, down, padding, groups, flip_weight)
        "up2_grouped_noflip": ([1, 2 * 6, 5, 5], [2 * 4, 6, 3, 3], 2, 1, 1, 2, False),   # fused conv0
        "same3x3_grouped": ([1, 2 * 6, 7, 7], [2 * 5, 6, 3, 3], 1, 1, 1, 2, True),       # fused conv1
        "conv1x1": ([2, 6, 5, 5], [3, 6, 1, 1], 1, 1, 0, 1, True),                        # torgb
        "up2_plain": ([2, 4, 4, 4], [5, 4, 3, 3], 2, 1, 1, 1, False),
        "down2": ([2, 4, 8, 8], [5, 4, 3, 3], 1, 2, 1, 1, True),
        "up2_1x1": ([1, 3, 4, 4], [2, 3, 1, 1], 2, 1, 0, 1, True),
    }
    for name, (xs, ws, up, down, pad, groups, flip) in cases.items():
        x = torch.randn(xs, generator=g).requires_grad_(True)
        w = torch.randn(ws, generator=g)
        y = ref_c2r.conv2d_resample(x, w, f=f4, up=up, down=down, padding=pad, groups=groups, flip_weight=flip)
        dy = torch.randn(y.shape, generator=g)
        (dx,) = torch.autograd.grad(y, x, dy)
        out.update({f"{name}/x": x, f"{name}/w": w, f"{name}/y": y, f"{name}/dy": dy, f"{name}/dx": dx,
                    f"{name}/meta": np.array([up, down, pad, groups, int(flip)])})
    out["f4"] = f4
    save("ops_conv2d_resample.npz", out)


# ---------------------------------------------------------------------------------- tiny generator on reference ops


class RefFC(torch.nn.Module):
    def __init__(self, fin, fout, bias_init=1.0):
        super().__init__()
        self.weight = torch.nn.Parameter(torch.randn(fout, fin))
        self.bias = torch.nn.Parameter(torch.full([fout], bias_init))
        self.weight_gain = 1 / np.sqrt(fin)

    def forward(self, x):
        return torch.addmm(self.bias.unsqueeze(0), x, (self.weight * self.weight_gain).t())


def ref_modconv(x, weight, styles, noise=None, up=1, padding=0, f=None, demodulate=True, flip_weight=True):
    """Upstream fused modulated_conv2d evaluated with the REFERENCE's conv2d_resample."""
    n = x.shape[0]
    oc, ic, kh, kw = weight.shape
    w = weight.unsqueeze(0) * styles.reshape(n, 1, -1, 1, 1)
    if demodulate:
        d = (w.square().sum(dim=[2, 3, 4]) + 1e-8).rsqrt()
        w = w * d.reshape(n, -1, 1, 1, 1)
    x = x.reshape(1, -1, *x.shape[2:])
    x = ref_c2r.conv2d_resample(x, w.reshape(-1, ic, kh, kw), f=f, up=up, padding=padding, groups=n,
                                flip_weight=flip_weight)
    x = x.reshape(n, -1, *x.shape[2:])
    if noise is not None:
        x = x.add_(noise)
    return x


class RefSynthesisLayer(torch.nn.Module):
    def __init__(self, cin, cout, res, up, conv_clamp):
        super().__init__()
        self.resolution, self.up, self.conv_clamp, self.padding = res, up, conv_clamp, 1
        self.activation = "lrelu"
        self.register_buffer("resample_filter", ref_upfirdn2d.setup_filter([1, 3, 3, 1]))
        self.affine = RefFC(512, cin)
        self.weight = torch.nn.Parameter(torch.randn(cout, cin, 3, 3))
        self.register_buffer("noise_const", torch.randn(res, res))
        self.noise_strength = torch.nn.Parameter(torch.zeros([]))
        self.bias = torch.nn.Parameter(torch.zeros(cout))

    def forward(self, x, w, noise_mode="const", fused_modconv=True, gain=1):
        s = self.affine(w)
        noise = self.noise_const * self.noise_strength if noise_mode == "const" else None
        x = ref_modconv(x, self.weight, s, noise=noise, up=self.up, padding=1, f=self.resample_filter,
                        flip_weight=(self.up == 1))
        return ref_bias_act.bias_act(x, self.bias, act="lrelu", gain=np.sqrt(2) * gain,
                                     clamp=self.conv_clamp * gain, impl="ref")


class RefToRGB(torch.nn.Module):
    def __init__(self, cin, conv_clamp):
        super().__init__()
        self.conv_clamp = conv_clamp
        self.affine = RefFC(512, cin)
        self.weight = torch.nn.Parameter(torch.randn(3, cin, 1, 1))
        self.bias = torch.nn.Parameter(torch.zeros(3))
        self.weight_gain = 1 / np.sqrt(cin)

    def forward(self, x, w, fused_modconv=True):
        s = self.affine(w) * self.weight_gain
        x = ref_modconv(x, self.weight, s, demodulate=False)
        return ref_bias_act.bias_act(x, self.bias, clamp=self.conv_clamp, impl="ref")


class RefBlock(torch.nn.Module):
    def __init__(self, cin, cout, res, conv_clamp):
        super().__init__()
        self.in_channels, self.w_dim, self.resolution, self.img_channels = cin, 512, res, 3
        self.is_last, self.architecture, self.use_fp16, self.channels_last = False, "skip", False, False
        self.register_buffer("resample_filter", ref_upfirdn2d.setup_filter([1, 3, 3, 1]))
        self.num_conv = 0
        if cin == 0:
            self.const = torch.nn.Parameter(torch.randn(cout, res, res))
        else:
            self.conv0 = RefSynthesisLayer(cin, cout, res, 2, conv_clamp)
            self.num_conv += 1
        self.conv1 = RefSynthesisLayer(cout, cout, res, 1, conv_clamp)
        self.num_conv += 1
        self.torgb = RefToRGB(cout, conv_clamp)
        self.num_torgb = 1


class RefG(torch.nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.synthesis = torch.nn.Module()
        res_log2 = int(np.log2(cfg["img_resolution"]))
        self.synthesis.block_resolutions = [2 ** i for i in range(2, res_log2 + 1)]
        ch = {r: min(cfg["channel_base"] // r, cfg["channel_max"]) for r in self.synthesis.block_resolutions}
        for r in self.synthesis.block_resolutions:
            setattr(self.synthesis, f"b{r}", RefBlock(ch[r // 2] if r > 4 else 0, ch[r], r, cfg["conv_clamp"]))


def gen_synthesis():
    out = {}
    for tag, res, cbase, clamp, n in (("r32", 32, 512, 256.0, 3), ("r16_clamp", 16, 256, 0.6, 2)):
        cfg = synthetic.generator_config(resolution=res, channel_base=cbase, conv_clamp=clamp)
        sd = {k: v for k, v in synthetic.generator_state_dict(cfg, seed=7).items() if k.startswith("synthesis.")}
        G = RefG(cfg).eval()
        missing = G.load_state_dict(sd, strict=False)
        assert not missing.unexpected_keys, missing.unexpected_keys
        assert all(k.endswith("resample_filter") for k in missing.missing_keys), missing.missing_keys
        temp_shapes = ref_utils.get_temp_shapes(G)
        styles = synthetic.synthetic_styles(n, seed=11).requires_grad_(True)
        until_k = len(G.synthesis.block_resolutions) - 1
        xs, img = ref_utils.generate_image(G, until_k, styles, temp_shapes, "const", "cpu")
        cot = torch.randn(img.shape, generator=torch.Generator().manual_seed(5))
        (dstyles,) = torch.autograd.grad((img * cot).sum(), styles)
        out[f"{tag}/meta"] = np.array([res, cbase, n, until_k])
        out[f"{tag}/clamp"] = np.array(clamp)
        out[f"{tag}/styles"] = styles
        out[f"{tag}/img"] = img
        out[f"{tag}/cot"] = cot
        out[f"{tag}/dstyles"] = dstyles
        out[f"{tag}/temp_shapes"] = np.array(temp_shapes)
        for k, x in enumerate(xs):
            out[f"{tag}/xs{k}"] = x
    save("synthesis_tiny.npz", out)


# ---------------------------------------------------------------------------------- loss nets


def gen_irse50():
    from id_loss.model_irse import Backbone
    net = Backbone(input_size=112, num_layers=50, drop_ratio=0.6, mode="ir_se").eval()
    net.load_state_dict(synthetic.seeded_state_dict(net, seed=3))
    g = torch.Generator().manual_seed(9)
    x = torch.randn([2, 3, 112, 112], generator=g).requires_grad_(True)
    y = net(x)
    cot = torch.randn(y.shape, generator=g)
    (dx,) = torch.autograd.grad(y, x, cot)
    save("irse50.npz", {"x": x, "y": y, "cot": cot, "dx": dx})


def gen_clip():
    from transformers import CLIPVisionConfig, CLIPVisionModelWithProjection
    from oracle.losses import CLIPVisual
    ours = CLIPVisual().eval()
    sd = synthetic.seeded_state_dict(ours, seed=4)
    cfg = CLIPVisionConfig(hidden_size=768, intermediate_size=3072, projection_dim=512, num_hidden_layers=12,
                           num_attention_heads=12, image_size=224, patch_size=32, hidden_act="quick_gelu",
                           layer_norm_eps=1e-5)
    hf = CLIPVisionModelWithProjection(cfg).eval()
    hsd = {}
    v = "vision_model."
    hsd[v + "embeddings.patch_embedding.weight"] = sd["conv1.weight"]
    hsd[v + "embeddings.class_embedding"] = sd["class_embedding"]
    hsd[v + "embeddings.position_embedding.weight"] = sd["positional_embedding"]
    hsd[v + "pre_layrnorm.weight"], hsd[v + "pre_layrnorm.bias"] = sd["ln_pre.weight"], sd["ln_pre.bias"]
    hsd[v + "post_layernorm.weight"], hsd[v + "post_layernorm.bias"] = sd["ln_post.weight"], sd["ln_post.bias"]
    hsd["visual_projection.weight"] = sd["proj"].t().contiguous()
    for i in range(12):
        o, h = f"transformer.resblocks.{i}.", f"{v}encoder.layers.{i}."
        qw, kw_, vw = sd[o + "attn.in_proj_weight"].chunk(3)
        qb, kb, vb = sd[o + "attn.in_proj_bias"].chunk(3)
        hsd[h + "self_attn.q_proj.weight"], hsd[h + "self_attn.q_proj.bias"] = qw, qb
        hsd[h + "self_attn.k_proj.weight"], hsd[h + "self_attn.k_proj.bias"] = kw_, kb
        hsd[h + "self_attn.v_proj.weight"], hsd[h + "self_attn.v_proj.bias"] = vw, vb
        hsd[h + "self_attn.out_proj.weight"] = sd[o + "attn.out_proj.weight"]
        hsd[h + "self_attn.out_proj.bias"] = sd[o + "attn.out_proj.bias"]
        for a, b in (("ln_1", "layer_norm1"), ("ln_2", "layer_norm2")):
            hsd[h + b + ".weight"], hsd[h + b + ".bias"] = sd[o + a + ".weight"], sd[o + a + ".bias"]
        hsd[h + "mlp.fc1.weight"], hsd[h + "mlp.fc1.bias"] = sd[o + "mlp.c_fc.weight"], sd[o + "mlp.c_fc.bias"]
        hsd[h + "mlp.fc2.weight"], hsd[h + "mlp.fc2.bias"] = sd[o + "mlp.c_proj.weight"], sd[o + "mlp.c_proj.bias"]
    res = hf.load_state_dict(hsd, strict=False)
    assert not res.unexpected_keys and all("position_ids" in k for k in res.missing_keys), res
    g = torch.Generator().manual_seed(12)
    x = torch.randn([2, 3, 224, 224], generator=g)
    with torch.no_grad():
        y = hf(pixel_values=x).image_embeds
    save("clip_vit_b32_hf.npz", {"x": x, "y": y})


if __name__ == "__main__":
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    which = sys.argv[1:] or ["upfirdn2d", "bias_act", "conv2d_resample", "synthesis", "irse50", "clip"]
    for w in which:
        globals()[f"gen_{w}"]()
