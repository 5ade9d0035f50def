"""Generate the golden vectors under tests/golden/ by running the REFERENCE's own code on CPU.

Run here (the container that has /root/reference), never on the GPU box:

    python tests/golden/make_golden.py

What is imported from the reference (read-only, CPU, its pure-torch ``_ref`` paths):
  torch_utils.ops.upfirdn2d / bias_act / conv2d_resample / fma, utils.block_forward /
  utils.generate_image / utils.get_temp_shapes (with a stub ``cv2`` module: cv2 is only used by the
  blending helpers), id_loss.model_irse.Backbone, legacy.convert_tf_generator (with the oracle Generator standing
  in for the absent training.networks).
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
sys.path.insert(0, HERE)
from fixture_inputs import LOSS_TEXT, block_sums, loss_inputs, probes  # noqa: E402

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


def gen_clip_text():
    """The oracle's CLIP text encoder vs transformers.CLIPTextModelWithProjection (causal mask, quick_gelu,
    EOS pooling) with the same seeded weights -- an architecture cross-check (openai/CLIP is absent)."""
    from transformers import CLIPTextConfig, CLIPTextModelWithProjection
    from oracle.losses import CLIPText
    ours = CLIPText().eval()
    sd = synthetic.seeded_state_dict(ours, seed=6)
    ours.load_state_dict(sd)
    cfg = CLIPTextConfig(vocab_size=49408, hidden_size=512, intermediate_size=2048, projection_dim=512,
                         num_hidden_layers=12, num_attention_heads=8, max_position_embeddings=77,
                         hidden_act="quick_gelu", layer_norm_eps=1e-5, eos_token_id=49407, bos_token_id=49406,
                         pad_token_id=0)
    hf = CLIPTextModelWithProjection(cfg).eval()
    t = "text_model."
    hsd = {t + "embeddings.token_embedding.weight": sd["token_embedding.weight"],
           t + "embeddings.position_embedding.weight": sd["positional_embedding"],
           t + "final_layer_norm.weight": sd["ln_final.weight"], t + "final_layer_norm.bias": sd["ln_final.bias"],
           "text_projection.weight": sd["text_projection"].t().contiguous()}
    for i in range(12):
        o, h = f"transformer.resblocks.{i}.", f"{t}encoder.layers.{i}."
        for n, (w, b) in zip(("q", "k", "v"), zip(sd[o + "attn.in_proj_weight"].chunk(3), sd[o + "attn.in_proj_bias"].chunk(3))):
            hsd[f"{h}self_attn.{n}_proj.weight"], hsd[f"{h}self_attn.{n}_proj.bias"] = w, b
        hsd[h + "self_attn.out_proj.weight"] = sd[o + "attn.out_proj.weight"]
        hsd[h + "self_attn.out_proj.bias"] = sd[o + "attn.out_proj.bias"]
        for a, b in (("ln_1", "layer_norm1"), ("ln_2", "layer_norm2")):
            hsd[h + b + ".weight"], hsd[h + b + ".bias"] = sd[o + a + ".weight"], sd[o + a + ".bias"]
        hsd[h + "mlp.fc1.weight"], hsd[h + "mlp.fc1.bias"] = sd[o + "mlp.c_fc.weight"], sd[o + "mlp.c_fc.bias"]
        hsd[h + "mlp.fc2.weight"], hsd[h + "mlp.fc2.bias"] = sd[o + "mlp.c_proj.weight"], sd[o + "mlp.c_proj.bias"]
    res = hf.load_state_dict(hsd, strict=False)
    assert not res.unexpected_keys and all("position_ids" in k for k in res.missing_keys), res
    g = torch.Generator().manual_seed(14)
    tokens = torch.zeros(3, 77, dtype=torch.long)
    for i, n in enumerate((5, 12, 75)):
        tokens[i, 0] = 49406
        tokens[i, 1:n + 1] = torch.randint(1, 49405, (n,), generator=g)
        tokens[i, n + 1] = 49407
    with torch.no_grad():
        y = hf(input_ids=tokens).text_embeds
        y_ours = ours(tokens)
    print("oracle vs HF text tower max |diff|", (y - y_ours).abs().max().item())
    save("clip_text_hf.npz", {"tokens": tokens, "y": y})


def gen_mapper():
    """latent_mappers.Mapper of the REFERENCE (latent_mappers.py:12-93, with e4e's PixelNorm from
    encoder4editing/models/stylegan2/model.py:10-15) on seeded weights; the e4e CUDA op package (JIT-built
    at import) and torchvision are import-only stubs -- the mapper never calls them."""
    tv = _stub("torchvision")
    tv.transforms = _stub("torchvision.transforms", Compose=_Absent, Resize=_Absent, CenterCrop=_Absent)
    _stub("encoder4editing.models.stylegan2.op", FusedLeakyReLU=_Absent, fused_leaky_relu=_Absent, upfirdn2d=_Absent)
    import latent_mappers as ref_lm
    out = {}
    for slope in (0.01, 0.2):
        m = ref_lm.Mapper(neg_slope=slope).eval()
        sd = synthetic.seeded_state_dict(m, seed=8)
        m.load_state_dict(sd)
        x = synthetic.synthetic_styles(3, seed=8)[:, [2, 3, 5, 6, 8, 9, 11, 12]]
        with torch.no_grad():
            y = m(x)
        out[f"s{slope}/y"] = y
    out["x"] = x
    save("mapper.npz", out)


# ---------------------------------------------------------------------------------- loss composition + loop


def _stub(name, **attrs):
    m = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules.setdefault(name, m)
    return m


class _Absent:
    """Placeholder for third-party / weight-loading names the reference imports but the path never calls."""

    def __init__(self, *a, **k):
        raise RuntimeError("import-only stub: not available offline")


def import_reference_losses():
    """Import the reference's find_direction / clip_loss / id_loss modules with IMPORT-ONLY stubs for what
    is absent offline (wandb, openai clip, torchvision, the landmark models).  Nothing stubbed is called on
    the loss path: CLIP's image encoder is supplied as an object (``_ClipModel``), IDLoss is built without
    its .pth, and the torchvision Resize+CenterCrop is passed in as ``transf`` (``bicubic_transf``)."""
    _stub("wandb", init=lambda *a, **k: None, log=lambda *a, **k: None, Image=_Absent)
    _stub("clip", load=_Absent, tokenize=_Absent)
    tv = _stub("torchvision")
    tv.transforms = _stub("torchvision.transforms", Compose=_Absent, Resize=_Absent, CenterCrop=_Absent)
    tv.models = _stub("torchvision.models")
    _stub("clip_loss_nada", CLIPLoss=_Absent)
    _stub("MTCNN", detect_faces=_Absent)
    _stub("mobilenet_facial", MobileNet_GDConv=_Absent)
    _stub("warp_images", crop_face=_Absent)
    import clip_loss as ref_clip_loss                           # clip_loss.py
    import find_direction as ref_fd                             # find_direction.py
    from id_loss import id_loss as ref_id_loss                  # id_loss/id_loss.py
    return ref_fd, ref_clip_loss, ref_id_loss


def bicubic_transf(x, size=224):
    """torchvision 0.8 tensor Resize(size, BICUBIC) + CenterCrop(size) on float input (functional_tensor:
    F.interpolate(mode='bicubic', align_corners=False), no antialias, no clamp for float dtypes)."""
    h, w = x.shape[-2:]
    nh, nw = (size, int(size * w / h)) if h <= w else (int(size * h / w), size)
    x = torch.nn.functional.interpolate(x, size=(nh, nw), mode="bicubic", align_corners=False)
    top, left = int(round((nh - size) / 2.0)), int(round((nw - size) / 2.0))
    return x[..., top:top + size, left:left + size]


class _ClipModel:
    """Stands in for the object ``clip.load`` returns: only ``encode_image`` is used by CLIPLoss.forward."""

    def __init__(self, visual):
        self.visual = visual

    def encode_image(self, image):
        return self.visual(image)


def ref_clip_loss_obj(ref_clip_loss, visual, text_features):
    """The reference CLIPLoss (clip_loss.py:7-34) without clip.load/encode_text: model + text direction set."""
    obj = ref_clip_loss.CLIPLoss.__new__(ref_clip_loss.CLIPLoss)
    torch.nn.Module.__init__(obj)
    obj.model = _ClipModel(visual)
    t = text_features.reshape(1, -1).float()
    obj.text_features = t / t.norm(dim=1, keepdim=True)
    return obj


def ref_id_loss_obj(ref_id_loss, seed=3):
    """The reference IDLoss (id_loss/id_loss.py:7-39) with a seeded Backbone instead of model_ir_se50.pth."""
    obj = ref_id_loss.IDLoss.__new__(ref_id_loss.IDLoss)
    torch.nn.Module.__init__(obj)
    obj.facenet = ref_id_loss.Backbone(input_size=112, num_layers=50, drop_ratio=0.6, mode="ir_se")
    obj.facenet.load_state_dict(synthetic.seeded_state_dict(obj.facenet, seed=seed))
    obj.facenet.eval().requires_grad_(False)
    obj.pool = torch.nn.AdaptiveAvgPool2d((256, 256))
    obj.face_pool = torch.nn.AdaptiveAvgPool2d((112, 112))
    obj.opts = "a"
    return obj


def seeded_visual(name, seed):
    from oracle.losses import CLIPVisual
    from stylemc_amd.clip_model import VIT_CONFIGS
    vis = CLIPVisual(**VIT_CONFIGS[name]).eval()
    vis.load_state_dict(synthetic.seeded_state_dict(vis, seed=seed))
    return vis.requires_grad_(False)


def gen_losses():
    """compute_loss / unprocess / CLIPLoss.forward / IDLoss.forward of the REFERENCE (find_direction.py:49-52,
    148-200; clip_loss.py:24-34; id_loss/id_loss.py:18-39) on seeded images at 512 px, clip_type small and
    double, landmarks coefficient 0.  Stored: the four loss terms, the total, and d total / d img as 8x8 block
    sums + 8 seeded probes (the inputs are regenerated from seeds by the tests)."""
    ref_fd, ref_cl, ref_il = import_reference_losses()
    T = ref_fd.S_TRAINABLE_SPACE_CHANNELS
    text = synthetic.text_direction(*LOSS_TEXT)
    idl = ref_id_loss_obj(ref_il)
    cl32 = ref_clip_loss_obj(ref_cl, seeded_visual("ViT-B/32", 4), text)
    cl16 = ref_clip_loss_obj(ref_cl, seeded_visual("ViT-B/16", 4), text)
    mean, std = ref_utils.get_mean_std("cpu")
    out = {}
    for clip_type in ("small", "double"):
        img, orig, styles, delta = loss_inputs()
        img.requires_grad_(True)
        sdir = torch.zeros(1, 26, 512)
        sdir[:, T] = delta
        styles2 = styles + sdir
        loss, parts = ref_fd.compute_loss(
            img, orig, bicubic_transf, mean, std, "cpu", "default", clip_type, 1.0, cl32,
            cl16 if clip_type == "double" else None, LOSS_TEXT[0], LOSS_TEXT[1], idl, 0.6, None, 0.0, None, 224,
            styles, styles2, 0.1)
        (dimg,) = torch.autograd.grad(loss, img)
        p = f"{clip_type}/"
        out[p + "loss"] = loss.detach()
        for k in ("clip_loss", "identity_loss", "l2_loss"):
            out[p + k] = torch.as_tensor(parts[k]).detach()
        out[p + "dimg_blocks8"] = block_sums(dimg, 8).float()
        out[p + "dimg_probes"] = probes(dimg)
        out[p + "unprocess_img"] = ref_fd.unprocess(img.detach(), bicubic_transf, mean, std)[:, :, ::8, ::8]
    save("loss_composition.npz", out)


class _Tok:
    """What the stubbed ``clip.tokenize`` returns: the strings themselves (E_T is a seeded per-string stand-in)."""

    def __init__(self, strings):
        self.strings = list(strings)

    def to(self, device):
        return self


class _NadaClipModel:
    """Stands in for the model ``clip.load`` returns to clip_loss_nada.CLIPLoss: encode_image = the seeded oracle
    ViT, encode_text = synthetic.text_embeddings (seeded E_T per string), and the openai/CLIP ``CLIP.forward``
    (normalise both, logit_scale.exp() * cos) restated for the global loss (third-party: parity unpinned)."""

    def __init__(self, visual, logit_scale):
        self.visual = visual
        self.logit_scale = torch.tensor(logit_scale, dtype=torch.float32)

    def encode_image(self, image):
        return self.visual(image)

    def encode_text(self, tokens):
        return synthetic.text_embeddings(tokens.strings)

    def __call__(self, image, tokens):
        i = self.encode_image(image)
        t = self.encode_text(tokens)
        i = i / i.norm(dim=1, keepdim=True)
        t = t / t.norm(dim=1, keepdim=True)
        logits = self.logit_scale.exp() * i @ t.t()
        return logits, logits.t()


def import_reference_nada():
    """The reference clip_loss_nada module with import-only stubs (clip, torchvision.transforms); must be imported
    before import_reference_losses() replaces it by a stub."""
    stub = sys.modules.get("clip_loss_nada")
    if stub is not None and getattr(stub, "__file__", None) is None:
        del sys.modules["clip_loss_nada"]
    clip = _stub("clip", load=_Absent, tokenize=_Absent)
    clip.tokenize = lambda strings: _Tok([strings] if isinstance(strings, str) else strings)
    tv = _stub("torchvision")
    tv.transforms = _stub("torchvision.transforms", Compose=_Absent, Resize=_Absent, CenterCrop=_Absent,
                          Normalize=_Absent)
    import clip_loss_nada as ref_nada                          # clip_loss_nada.py
    return ref_nada


def nada_preprocess_transf(x):
    """clip_loss_nada.py:72-75 preprocess: torchvision Normalize(-1, 2) (sub_ then div_), the CLIP preprocess'
    Resize(224, BICUBIC) + CenterCrop(224) (bicubic_transf), CLIP Normalize -- restated (torchvision / clip absent)."""
    mean, std = ref_utils.get_mean_std("cpu")
    return (bicubic_transf((x - (-1.0)) / 2.0) - mean) / std


def ref_nada_obj(ref_nada, visual, lambda_direction=1.0, lambda_global=0.0, lambda_manifold=0.0):
    """The reference clip_loss_nada.CLIPLoss (:62-101) without clip.load: model / preprocess / losses set."""
    import math
    obj = ref_nada.CLIPLoss.__new__(ref_nada.CLIPLoss)
    torch.nn.Module.__init__(obj)
    obj.device = "cpu"
    obj.model = _NadaClipModel(visual, math.log(100.0))
    obj.clip_preprocess = None
    obj.preprocess = nada_preprocess_transf
    obj.target_direction = None
    obj.patch_text_directions = None
    obj.patch_loss = ref_nada.DirectionLoss("mae")
    obj.direction_loss = ref_nada.DirectionLoss("cosine")
    obj.patch_direction_loss = torch.nn.CosineSimilarity(dim=2)
    obj.lambda_global, obj.lambda_patch, obj.lambda_direction = lambda_global, 0.0, lambda_direction
    obj.lambda_manifold, obj.lambda_texture = lambda_manifold, 0.0
    obj.src_text_features = None
    obj.target_text_features = None
    obj.angle_loss = torch.nn.L1Loss()
    return obj


NADA_CASES = {"nada": dict(lambda_direction=1.0), "nada_global": dict(lambda_direction=0.0, lambda_global=1.0),
              "mix": dict(lambda_direction=1.0, lambda_global=0.5, lambda_manifold=0.7)}


def gen_nada():
    """clip_loss_nada.CLIPLoss.forward of the REFERENCE (clip_loss_nada.py:117-229,324-346: template text direction,
    directional / global / angle losses) on seeded 512-px images, and find_direction.compute_loss with
    --clip_loss_type nada / nada_global, clip_type small and double (find_direction.py:100-114,150-157,172-200)."""
    ref_nada = import_reference_nada()
    ref_fd, ref_cl, ref_il = import_reference_losses()
    T = ref_fd.S_TRAINABLE_SPACE_CHANNELS
    out = {}
    src_class, tgt_class = LOSS_TEXT[1], LOSS_TEXT[0]
    for case, kw in NADA_CASES.items():
        obj = ref_nada_obj(ref_nada, seeded_visual("ViT-B/32", 4), **kw)
        img, orig, _, _ = loss_inputs()
        img.requires_grad_(True)
        loss = obj(orig, src_class, img, tgt_class)
        (dimg,) = torch.autograd.grad(loss, img)
        p = f"forward/{case}/"
        out[p + "loss"] = loss.detach()
        out[p + "dimg_blocks8"] = block_sums(dimg, 8).float()
        out[p + "dimg_probes"] = probes(dimg)
        if obj.target_direction is not None:
            out[p + "target_direction"] = obj.target_direction
    out["preprocess_img"] = nada_preprocess_transf(loss_inputs()[0])[:, :, ::8, ::8]
    idl = ref_id_loss_obj(ref_il)
    mean, std = ref_utils.get_mean_std("cpu")
    for clip_loss_type in ("nada", "nada_global"):
        kw = NADA_CASES[clip_loss_type]
        for clip_type in ("small", "double"):
            cl1 = ref_nada_obj(ref_nada, seeded_visual("ViT-B/32", 4), **kw)
            cl2 = ref_nada_obj(ref_nada, seeded_visual("ViT-B/16", 4), **kw) if clip_type == "double" else None
            img, orig, styles, delta = loss_inputs()
            img.requires_grad_(True)
            sdir = torch.zeros(1, 26, 512)
            sdir[:, T] = delta
            loss, parts = ref_fd.compute_loss(
                img, orig, bicubic_transf, mean, std, "cpu", clip_loss_type, clip_type, 1.0, cl1, cl2, LOSS_TEXT[0],
                LOSS_TEXT[1], idl, 0.6, None, 0.0, None, 224, styles, styles + sdir, 0.1)
            (dimg,) = torch.autograd.grad(loss, img)
            p = f"{clip_loss_type}/{clip_type}/"
            out[p + "loss"] = loss.detach()
            for k in ("clip_loss", "identity_loss", "l2_loss"):
                out[p + k] = torch.as_tensor(parts[k]).detach()
            out[p + "dimg_blocks8"] = block_sums(dimg, 8).float()
            out[p + "dimg_probes"] = probes(dimg)
    save("loss_nada.npz", out)


def gen_styles():
    """utils.split_ws / utils.get_styles of the REFERENCE (utils.py:77-87,123-158) on a small generator (b4 must
    be 512 wide: utils.py:135 writes the b4 row at full width)."""
    cfg = synthetic.generator_config(resolution=32, channel_base=2048, conv_clamp=256.0)
    sd = {k: v for k, v in synthetic.generator_state_dict(cfg, seed=7).items() if k.startswith("synthesis.")}
    G = RefG(cfg).eval()
    G.load_state_dict(sd, strict=False)
    G.synthesis.w_dim = 512
    G.synthesis.num_ws = sum(getattr(G.synthesis, f"b{r}").num_conv for r in G.synthesis.block_resolutions) + 1
    ws = torch.randn(3, G.synthesis.num_ws, 512, generator=torch.Generator().manual_seed(13))
    block_ws = ref_utils.split_ws(G, ws)
    styles, shapes = ref_utils.get_styles(G, ws, block_ws, "cpu")
    save("styles_from_w.npz", {"ws": ws, "styles": styles, "temp_shapes": np.array(shapes)})


def config1_problem():
    """BASELINE config 1: paper256 FFHQ-256 generator (channel_base 16384), S codes of seeds 1-4 through the
    mapping (psi 0.7, generate_w.py:48-50) and the reference get_styles, bs 1, 4 epochs, clip_type small."""
    from oracle import networks as ON
    cfg = synthetic.generator_config(resolution=256)
    assert cfg["channel_base"] == 16384
    sd = synthetic.generator_state_dict(cfg, seed=0)
    Go = ON.Generator(512, 0, 512, 256, 3, channel_base=cfg["channel_base"], conv_clamp=cfg["conv_clamp"])
    Go.load_state_dict(sd, strict=False)
    with torch.no_grad():
        ws = Go.eval().mapping(synthetic.seed_latents([1, 2, 3, 4]), None, truncation_psi=0.7)
    return cfg, sd, ws


def gen_config1():
    """The REFERENCE's hot loop (find_direction.py:292-339, statement for statement; the click/wandb/landmark
    plumbing left out) on config 1, driven by the reference's generate_image / compute_loss / CLIPLoss /
    IDLoss and a torch SGD, from the seeded start direction passed the way --resume passes one (:266-271)."""
    import math
    ref_fd, ref_cl, ref_il = import_reference_losses()
    from stylemc_amd.find_direction import initial_delta
    T = ref_fd.S_TRAINABLE_SPACE_CHANNELS
    cfg, sd, ws = config1_problem()
    G = RefG(cfg).eval()
    G.load_state_dict({k: v for k, v in sd.items() if k.startswith("synthesis.")}, strict=False)
    G.synthesis.w_dim = 512
    G.synthesis.num_ws = ws.shape[1]
    G.requires_grad_(False)
    # get_styles turns every affine into Identity and returns the same widths get_temp_shapes would
    # (w_s_converter.py and find_direction.py load G separately)
    styles_array, temp_shapes = ref_utils.get_styles(G, ws, ref_utils.split_ws(G, ws), "cpu")
    mean, std = ref_utils.get_mean_std("cpu")
    text = synthetic.text_direction(*LOSS_TEXT)
    idl = ref_id_loss_obj(ref_il)
    cl = ref_clip_loss_obj(ref_cl, seeded_visual("ViT-B/32", 4), text)
    resolution, batch_size, learning_rate, n_epochs, seed = 256, 1, 1.5, 4, 2
    styles_direction = torch.zeros(1, 26, 512)
    styles_direction[:, T] = initial_delta(0, 0.01)
    start = styles_direction.clone()
    trainable_delta_s = styles_direction.index_select(1, torch.tensor(T))
    trainable_delta_s.requires_grad = True
    opt = torch.optim.SGD([trainable_delta_s], lr=learning_rate)
    n_items = styles_array.size(0)
    num_batches = math.ceil(n_items / batch_size)
    total = num_batches * n_epochs
    np.random.seed(seed)
    it = 0
    log = []
    for _ in range(n_epochs):
        for _ in range(num_batches):
            opt.zero_grad()
            it += 1
            lr = np.cos(np.pi * it / total) * learning_rate * 0.5 + learning_rate * 0.5
            for group in opt.param_groups:
                group["lr"] = lr
            i = np.random.randint(0, math.ceil(n_items / batch_size))
            styles = styles_array[i * batch_size:(i + 1) * batch_size]
            styles_direction[:, T] = trainable_delta_s
            styles2 = styles + styles_direction
            _, img = ref_utils.generate_image(G, {256: 6, 512: 7, 1024: 8}[resolution], styles2, temp_shapes,
                                              "const", "cpu")
            _, original_img = ref_utils.generate_image(G, {256: 6, 512: 7, 1024: 8}[resolution], styles,
                                                       temp_shapes, "const", "cpu")
            loss, parts = ref_fd.compute_loss(
                img, original_img, bicubic_transf, mean, std, "cpu", "default", "small", 1.0, cl, None,
                LOSS_TEXT[0], LOSS_TEXT[1], idl, 0.6, None, 0.0, None, 224, styles, styles2, 0.1)
            loss.backward(retain_graph=True)
            grad_norm = trainable_delta_s.grad.data.norm()
            opt.step()
            log.append([it, i, lr, float(loss), float(parts["clip_loss"]), float(parts["identity_loss"]),
                        float(parts["l2_loss"]), float(grad_norm)])
            print(log[-1])
    save("config1_direction.npz", {"s": styles_direction.detach(), "delta_final": trainable_delta_s.detach(),
                                   "start": start, "styles": styles_array, "ws": ws, "log": np.array(log),
                                   "meta": np.array([resolution, batch_size, n_epochs, seed])})


MAPPER_SUBSAMPLE = 61   # every 61st parameter element is stored (the mapper has 5.3 M parameters)


def flat_params(module):
    return torch.cat([p.detach().reshape(-1) for p in module.parameters()])


def gen_mapper_train():
    """The REFERENCE's train_latent_mapper loop (train_latent_mapper.py:138-196, statement for statement; click /
    wandb / landmark plumbing left out) on BASELINE config 1's problem (paper256 FFHQ-256, S codes of seeds 1-4),
    batch 2, 2 epochs (4 iterations), the script's defaults (lr 0.0005, identity 0.3, l2 0.8, clip 2.0, clip_type
    small), driven by the reference's Mapper, generate_image and compute_loss and torch Adam, from a seeded mapper
    passed the way --resume passes one (:118-120).  Stored: the per-iteration log, and the parameter update and the
    first iteration's gradient as per-tensor norms + every MAPPER_SUBSAMPLE-th element."""
    import math
    tv = _stub("torchvision")
    tv.transforms = _stub("torchvision.transforms", Compose=_Absent, Resize=_Absent, CenterCrop=_Absent)
    _stub("encoder4editing.models.stylegan2.op", FusedLeakyReLU=_Absent, fused_leaky_relu=_Absent, upfirdn2d=_Absent)
    import latent_mappers as ref_lm
    ref_fd, ref_cl, ref_il = import_reference_losses()
    T = ref_fd.S_TRAINABLE_SPACE_CHANNELS
    cfg, sd, ws = config1_problem()
    G = RefG(cfg).eval()
    G.load_state_dict({k: v for k, v in sd.items() if k.startswith("synthesis.")}, strict=False)
    G.synthesis.w_dim = 512
    G.synthesis.num_ws = ws.shape[1]
    G.requires_grad_(False)
    styles_array, temp_shapes = ref_utils.get_styles(G, ws, ref_utils.split_ws(G, ws), "cpu")
    mean, std = ref_utils.get_mean_std("cpu")
    idl = ref_id_loss_obj(ref_il)
    cl = ref_clip_loss_obj(ref_cl, seeded_visual("ViT-B/32", 4), synthetic.text_direction(*LOSS_TEXT))
    resolution, batch_size, learning_rate, n_epochs, seed, neg_slope = 256, 2, 0.0005, 2, 3, 0.01
    mapper = ref_lm.Mapper(neg_slope)
    mapper.load_state_dict(synthetic.seeded_state_dict(mapper, seed=8))
    start = flat_params(mapper).clone()
    opt = torch.optim.Adam(mapper.parameters(), lr=learning_rate, betas=(0.9, 0.999))
    n_items = styles_array.size(0)
    num_batches = math.ceil(n_items / batch_size)
    total = num_batches * n_epochs
    np.random.seed(seed)
    it = 0
    log, grad0 = [], None
    for _ in range(n_epochs):
        for _ in range(num_batches):
            opt.zero_grad()
            it += 1
            lr = np.cos(np.pi * it / total) * learning_rate * 0.5 + learning_rate * 0.5
            for group in opt.param_groups:
                group["lr"] = lr
            i = np.random.randint(0, math.ceil(n_items / batch_size))
            styles = styles_array[i * batch_size:(i + 1) * batch_size]
            delta = mapper(styles[:, T, :])
            styles2 = styles.clone()
            styles2[:, T] += delta
            _, img = ref_utils.generate_image(G, {256: 6, 512: 7, 1024: 8}[resolution], styles2, temp_shapes, "const",
                                              "cpu")
            _, original_img = ref_utils.generate_image(G, {256: 6, 512: 7, 1024: 8}[resolution], styles, temp_shapes,
                                                       "const", "cpu")
            loss, parts = ref_fd.compute_loss(
                img, original_img, bicubic_transf, mean, std, "cpu", "default", "small", 2.0, cl, None,
                LOSS_TEXT[0], LOSS_TEXT[1], idl, 0.3, None, 0.0, None, 224, styles, styles2, 0.8)
            loss.backward(retain_graph=True)
            grad_norm = sum(p.grad.data.norm() for p in mapper.parameters() if p.grad is not None)
            if grad0 is None:
                grad0 = torch.cat([p.grad.detach().reshape(-1) for p in mapper.parameters()])
            opt.step()
            log.append([it, i, lr, float(loss), float(parts["clip_loss"]), float(parts["identity_loss"]),
                        float(parts["l2_loss"]), float(grad_norm)])
            print(log[-1])
    update = flat_params(mapper) - start
    sizes = np.array([p.numel() for p in mapper.parameters()])
    bounds = np.concatenate([[0], np.cumsum(sizes)])
    save("mapper_train.npz", {
        "log": np.array(log), "meta": np.array([resolution, batch_size, n_epochs, seed]),
        "meta_f": np.array([learning_rate, neg_slope]), "styles": styles_array,
        "update_sub": update[::MAPPER_SUBSAMPLE], "grad0_sub": grad0[::MAPPER_SUBSAMPLE],
        "update_norms": np.array([update[a:b].norm().item() for a, b in zip(bounds[:-1], bounds[1:])]),
        "grad0_norms": np.array([grad0[a:b].norm().item() for a, b in zip(bounds[:-1], bounds[1:])]),
        "param_names": np.array([n for n, _ in mapper.named_parameters()])})


# ---------------------------------------------------------------------------------- TF-era network pickles


def tf_generator_tree():
    """A seeded synthetic TensorFlow-era StyleGAN2 G (the dnnlib.tflib Network state: version, static_kwargs, own
    variables, components): the config-f skip architecture at 32 px with fmap_base 256 and fmap_max 64 (channels
    64 / 64 / 32 / 16: every width the HIP kernels take), a 32-wide latent and 2 mapping layers so the fixture stays
    small.  Returns {component: [(name, array)]} with
    component '' (G: dlatent_avg), 'mapping', 'synthesis', and the static kwargs."""
    rng = np.random.RandomState(31)
    kw = dict(latent_size=32, dlatent_size=32, label_size=0, resolution=32, num_channels=3, mapping_layers=2,
              fmap_base=256, fmap_max=64, truncation_psi=0.5)
    R, zd, wd = 32, 32, 32
    ch = {r: min(kw["fmap_base"] * 2 // r, kw["fmap_max"]) for r in (4, 8, 16, 32)}

    def a(*shape):
        return rng.standard_normal(shape).astype(np.float32)

    mapping = []
    for i in range(kw["mapping_layers"]):
        mapping += [(f"Dense{i}/weight", a(zd if i == 0 else wd, wd)), (f"Dense{i}/bias", a(wd))]
    syn = [("4x4/Const/const", a(1, ch[4], 4, 4))]

    def layer(prefix, cin, cout, k=3):
        return [(f"{prefix}/weight", a(k, k, cin, cout)), (f"{prefix}/mod_weight", a(wd, cin)),
                (f"{prefix}/mod_bias", a(cin)), (f"{prefix}/bias", a(cout))]

    syn += layer("4x4/Conv", ch[4], ch[4]) + [("4x4/Conv/noise_strength", a())]
    syn += layer("4x4/ToRGB", ch[4], 3, k=1)
    for r in (8, 16, 32):
        syn += layer(f"{r}x{r}/Conv0_up", ch[r // 2], ch[r]) + [(f"{r}x{r}/Conv0_up/noise_strength", a())]
        syn += layer(f"{r}x{r}/Conv1", ch[r], ch[r]) + [(f"{r}x{r}/Conv1/noise_strength", a())]
        syn += layer(f"{r}x{r}/ToRGB", ch[r], 3, k=1)
    for k in range(2 * int(np.log2(R)) - 3):
        r = 2 ** ((k + 5) // 2)
        syn.append((f"noise{k}", a(1, 1, r, r)))
    return {"": [("dlatent_avg", a(wd))], "mapping": mapping, "synthesis": syn}, kw


def gen_tf_legacy():
    """The REFERENCE's legacy.convert_tf_generator (legacy.py:110-204) on tf_generator_tree(), with the oracle
    Generator standing in for the absent training.networks (as RefG does for the synthesis fixtures): the TF
    variables in, the converted G's every parameter and buffer out as shape + sha256 of its float32 bytes (bit-exact
    target of stylemc_amd.legacy), and the converted generator's image on fixed latents."""
    import json
    from oracle import networks as ON

    class StandInGenerator(ON.Generator):
        def __init__(self, z_dim, c_dim, w_dim, img_resolution, img_channels, mapping_kwargs=None,
                     synthesis_kwargs=None):
            mk = dict(mapping_kwargs or {})
            assert mk.pop("embed_features") is None and mk.pop("layer_features") is None
            assert mk.pop("activation") == "lrelu"
            super().__init__(z_dim, c_dim, w_dim, img_resolution, img_channels, mapping_kwargs=mk,
                             **dict(synthesis_kwargs or {}))

    tr = _stub("training")
    tr.networks = _stub("training.networks", Generator=StandInGenerator)
    import legacy as ref_legacy                                 # legacy.py
    tree, kw = tf_generator_tree()

    def net(comp):
        n = ref_legacy._TFNetworkStub()
        n.version, n.name, n.static_kwargs = 4, comp or "G", dict(kw) if comp == "" else {}
        n.variables = list(tree[comp])
        n.components = {}
        return n

    tf_G = net("")
    tf_G.components = {"mapping": net("mapping"), "synthesis": net("synthesis")}
    G = ref_legacy.convert_tf_generator(tf_G)
    out = {"static_kwargs": np.array(json.dumps(kw))}
    for comp, vs in tree.items():
        out[f"tf_names:{comp}"] = np.array([n for n, _ in vs])
        for n, v in vs:
            out[f"tf:{comp}:{n}"] = v
    import hashlib
    for n, t in list(G.named_parameters()) + list(G.named_buffers()):   # bit-exact target: shape + sha256 of the bytes
        a = np.ascontiguousarray(t.detach().numpy().astype(np.float32))
        out[f"sd:{n}"] = np.array([hashlib.sha256(a.tobytes()).hexdigest()] + [str(d) for d in a.shape])
    # the converted generator's output on fixed latents (the oracle layers): the GPU test renders the same
    z = torch.from_numpy(np.random.RandomState(32).standard_normal((2, 32)).astype(np.float32))
    with torch.no_grad():
        out["z"] = z
        out["img"] = G(z, None, truncation_psi=0.7, noise_mode="const")
    save("tf_legacy.npz", out)


if __name__ == "__main__":
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    which = sys.argv[1:] or ["upfirdn2d", "bias_act", "conv2d_resample", "synthesis", "irse50", "clip", "nada",
                             "losses", "styles", "config1", "mapper_train", "tf_legacy"]
    for w in which:
        globals()[f"gen_{w}"]()
