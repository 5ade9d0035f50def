"""Pin the CPU oracle against golden vectors produced by the reference's own code (CPU, no GPU)."""
import numpy as np
import pytest
import torch

from oracle import losses as O_loss
from oracle import networks as O_net
from oracle import ops as O
from oracle import synthesis as O_syn
from stylemc_amd import synthetic

CASES_UFD = ["blur_conv0", "up2_img", "down2_adj", "blur_adj", "rect_up2_down1", "crop_neg_pad", "odd_filter",
             "sep_filter8", "up4_down3", "single_pixel"]


def t(a):
    return torch.from_numpy(np.asarray(a))


@pytest.mark.parametrize("case", CASES_UFD)
def test_upfirdn2d_golden(golden, case):
    g = golden("ops_upfirdn2d.npz")
    p = lambda k: g[f"{case}/{k}"]
    x = t(p("x")).requires_grad_(True)
    up, down = [int(v) for v in p("up")], [int(v) for v in p("down")]
    y = O.upfirdn2d(x, t(p("f")), up=up, down=down, padding=[int(v) for v in p("pad")],
                    flip_filter=bool(p("flip")), gain=float(p("gain")))
    np.testing.assert_allclose(y.detach().numpy(), p("y"), rtol=1e-5, atol=1e-5)
    (dx,) = torch.autograd.grad(y, x, t(p("dy")))
    np.testing.assert_allclose(dx.numpy(), p("dx"), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("case", CASES_UFD)
def test_upfirdn2d_adjoint_rule(golden, case):
    """The reference's backward (upfirdn2d.py:245-261) = upfirdn2d with up/down swapped + flip."""
    g = golden("ops_upfirdn2d.npz")
    p = lambda k: g[f"{case}/{k}"]
    f = t(p("f"))
    if f.ndim != 2:
        pytest.skip("separable filters use two 1-D passes")
    x, dy = t(p("x")), t(p("dy"))
    up, down = [int(v) for v in p("up")], [int(v) for v in p("down")]
    pad = [int(v) for v in p("pad")]
    adj = O.upfirdn2d_adjoint_padding(x.shape[2], x.shape[3], dy.shape[2], dy.shape[3], f.shape[0], f.shape[1],
                                      up, down, pad)
    dx = O.upfirdn2d(dy, f, up=down, down=up, padding=adj, flip_filter=not bool(p("flip")), gain=float(p("gain")))
    np.testing.assert_allclose(dx.numpy(), p("dx"), rtol=1e-5, atol=1e-5)


def test_resample_helpers_golden(golden):
    g = golden("ops_upfirdn2d.npz")
    x, f = t(g["helper/x"]), t(g["helper/f4"])
    np.testing.assert_allclose(O.setup_filter([1, 3, 3, 1]).numpy(), g["helper/f4"], rtol=0, atol=0)
    np.testing.assert_allclose(O.upsample2d(x, f).numpy(), g["helper/upsample2d"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(O.downsample2d(x, f).numpy(), g["helper/downsample2d"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(O.filter2d(x, f).numpy(), g["helper/filter2d"], rtol=1e-6, atol=1e-6)


ACTS = ["linear", "relu", "lrelu", "tanh", "sigmoid", "elu", "selu", "softplus", "swish"]


@pytest.mark.parametrize("act", ACTS)
@pytest.mark.parametrize("clamp", [None, 0.7])
def test_bias_act_golden(golden, act, clamp):
    g = golden("ops_bias_act.npz")
    name = f"{act}_c{'none' if clamp is None else clamp}"
    x = t(g[f"{name}/x"]).requires_grad_(True)
    b = t(g[f"{name}/b"]).requires_grad_(True)
    y = O.bias_act(x, b, act=act, clamp=clamp)
    np.testing.assert_allclose(y.detach().numpy(), g[f"{name}/y"], rtol=1e-6, atol=1e-6)
    dx, db = torch.autograd.grad(y, [x, b], t(g[f"{name}/dy"]))
    np.testing.assert_allclose(dx.numpy(), g[f"{name}/dx"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(db.numpy(), g[f"{name}/db"], rtol=1e-5, atol=1e-5)
    if act in ("linear", "relu", "lrelu"):
        # CUDA-kernel backward semantics (mask on the clamped output) agree off the measure-zero boundary.
        dxk = O.bias_act_grad(t(g[f"{name}/dy"]), y.detach(), act=act, clamp=clamp)
        np.testing.assert_allclose(dxk.numpy(), g[f"{name}/dx"], rtol=1e-5, atol=1e-6)


def test_bias_act_dim_gain_alpha(golden):
    g = golden("ops_bias_act.npz")
    y = O.bias_act(t(g["dim0/x"]), t(g["dim0/b"]), dim=0, act="lrelu", alpha=0.1, gain=3.0, clamp=2.0)
    np.testing.assert_allclose(y.numpy(), g["dim0/y"], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("case", ["up2_grouped_noflip", "same3x3_grouped", "conv1x1", "up2_plain", "down2", "up2_1x1"])
def test_conv2d_resample_golden(golden, case):
    g = golden("ops_conv2d_resample.npz")
    up, down, pad, groups, flip = [int(v) for v in g[f"{case}/meta"]]
    x = t(g[f"{case}/x"]).requires_grad_(True)
    y = O.conv2d_resample(x, t(g[f"{case}/w"]), f=t(g["f4"]), up=up, down=down, padding=pad, groups=groups,
                          flip_weight=bool(flip))
    np.testing.assert_allclose(y.detach().numpy(), g[f"{case}/y"], rtol=1e-5, atol=1e-5)
    (dx,) = torch.autograd.grad(y, x, t(g[f"{case}/dy"]))
    np.testing.assert_allclose(dx.numpy(), g[f"{case}/dx"], rtol=1e-5, atol=1e-5)


def oracle_G(res, cbase, clamp, seed=7):
    cfg = synthetic.generator_config(resolution=res, channel_base=cbase, conv_clamp=clamp)
    syn = O_net.SynthesisNetwork(w_dim=512, img_resolution=res, img_channels=3, channel_base=cbase,
                                 conv_clamp=clamp)
    sd = {k[len("synthesis."):]: v for k, v in synthetic.generator_state_dict(cfg, seed=seed).items()
          if k.startswith("synthesis.")}
    res_ = syn.load_state_dict(sd, strict=False)
    assert not res_.unexpected_keys and all(k.endswith("resample_filter") for k in res_.missing_keys)
    G = torch.nn.Module()
    G.synthesis = syn.eval()
    return G


@pytest.mark.parametrize("tag,fused", [("r32", True), ("r32", False), ("r16_clamp", True)])
def test_synthesis_golden(golden, tag, fused):
    """oracle block_forward/generate_image + restated layers vs the reference utils driving reference ops."""
    g = golden("synthesis_tiny.npz")
    res, cbase, n, until_k = [int(v) for v in g[f"{tag}/meta"]]
    G = oracle_G(res, cbase, float(g[f"{tag}/clamp"]))
    shapes = O_syn.get_temp_shapes(G)
    assert [tuple(s) for s in g[f"{tag}/temp_shapes"]] == shapes
    styles = t(g[f"{tag}/styles"]).requires_grad_(True)
    x = img = None
    row = 0
    xs = []
    for k, r in enumerate(G.synthesis.block_resolutions):
        block = getattr(G.synthesis, f"b{r}")
        width = 2 if r == 4 else 3
        x, img = O_syn.block_forward(block, x, img, styles[:, row:row + width], shapes[k], noise_mode="const",
                                     fused_modconv=fused)
        row += width
        xs.append(x)
    for k, xk in enumerate(xs):
        np.testing.assert_allclose(xk.detach().numpy(), g[f"{tag}/xs{k}"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(img.detach().numpy(), g[f"{tag}/img"], rtol=1e-4, atol=1e-4)
    (ds,) = torch.autograd.grad((img * t(g[f"{tag}/cot"])).sum(), styles)
    ref = g[f"{tag}/dstyles"]
    np.testing.assert_allclose(ds.numpy(), ref, rtol=1e-3, atol=1e-4 * np.abs(ref).max())


def test_generate_image_driver_golden(golden):
    g = golden("synthesis_tiny.npz")
    res, cbase, n, until_k = [int(v) for v in g["r32/meta"]]
    G = oracle_G(res, cbase, float(g["r32/clamp"]))
    shapes = O_syn.get_temp_shapes(G)
    xs, img = O_syn.generate_image(G, until_k, t(g["r32/styles"]), shapes, "const")
    np.testing.assert_allclose(img.detach().numpy(), g["r32/img"], rtol=1e-4, atol=1e-4)
    assert len(xs) == until_k + 1


def test_irse50_golden(golden):
    g = golden("irse50.npz")
    net = O_loss.IRSE50().eval()
    net.load_state_dict(synthetic.seeded_state_dict(net, seed=3))
    x = t(g["x"]).requires_grad_(True)
    y = net(x)
    np.testing.assert_allclose(y.detach().numpy(), g["y"], rtol=1e-4, atol=1e-5)
    (dx,) = torch.autograd.grad(y, x, t(g["cot"]))
    np.testing.assert_allclose(dx.numpy(), g["dx"], rtol=1e-3, atol=1e-3 * np.abs(g["dx"]).max())


def test_clip_visual_vs_hf_standin(golden):
    """Architecture cross-check only (openai/CLIP is absent: parity unpinned vs the reference)."""
    g = golden("clip_vit_b32_hf.npz")
    net = O_loss.CLIPVisual().eval()
    net.load_state_dict(synthetic.seeded_state_dict(net, seed=4))
    with torch.no_grad():
        y = net(t(g["x"]))
    np.testing.assert_allclose(y.numpy(), g["y"], rtol=1e-4, atol=1e-4)
