"""Parity of the HIP kernels (through the C ABI) against golden vectors and the CPU oracle.

Tolerances (fp32, different summation order than the reference's CPU path):
  elementwise ops: rtol 1e-5; FIR: atol 1e-5 relative to max|y|; modconv forward 2e-5 and backward
  1e-4 of the tensor's max magnitude; whole-network image 1e-4, style gradients 1e-3 (relative to
  max |grad|).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def t(a, dev="cpu"):
    return torch.from_numpy(np.asarray(a)).to(dev)


def close(a, b, tol, what=""):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu() if torch.is_tensor(b) else torch.from_numpy(np.asarray(b)).double()
    scale = max(b.abs().max().item(), 1e-12)
    err = (a - b).abs().max().item()
    assert err <= tol * scale, f"{what}: max err {err:.3e} > {tol:.1e} * {scale:.3e}"


def close_grad(a, b, tol, what="", max_flips=2):
    """Gradient through lrelu/clamp: the activation mask is discontinuous, so an element whose
    pre-activation sits within fp32 rounding of a kink (0, +-clamp) may legitimately take the other
    branch (GPU and CPU accumulate the conv in different orders).  Those isolated elements are allowed
    (at most `max_flips`, each still bounded by 1e-2 of the max); everything else must meet `tol`,
    and the whole tensor must agree to `tol` in relative Frobenius norm."""
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    scale = max(b.abs().max().item(), 1e-12)
    err = (a - b).abs()
    bad = int((err > tol * scale).sum())
    assert bad <= max_flips, f"{what}: {bad} elements beyond {tol:.1e} * {scale:.3e} (max {err.max():.3e})"
    assert err.max().item() <= 1e-2 * scale, f"{what}: max err {err.max():.3e}"
    rel = ((a - b).norm() / max(b.norm().item(), 1e-30)).item()
    assert rel <= tol, f"{what}: relative norm error {rel:.3e} > {tol:.1e}"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from stylemc_amd import build
    build.build(verbose=False)
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False


ACTS = ["linear", "relu", "lrelu", "tanh", "sigmoid", "elu", "selu", "softplus", "swish"]


@pytest.mark.parametrize("act", ACTS)
@pytest.mark.parametrize("clamp", [None, 0.7])
def test_bias_act_golden(golden, act, clamp):
    from stylemc_amd.torch_utils.ops import bias_act
    g = golden("ops_bias_act.npz")
    name = f"{act}_c{'none' if clamp is None else clamp}"
    x = t(g[f"{name}/x"], DEV).requires_grad_(True)
    b = t(g[f"{name}/b"], DEV).requires_grad_(True)
    y = bias_act.bias_act(x, b, act=act, clamp=clamp)
    close(y, g[f"{name}/y"], 1e-5, f"{name} y")
    dx, db = torch.autograd.grad(y, [x, b], t(g[f"{name}/dy"], DEV))
    close(dx, g[f"{name}/dx"], 1e-5, f"{name} dx")
    close(db, g[f"{name}/db"], 1e-5, f"{name} db")


def test_bias_act_second_order_and_dim():
    from oracle import ops as O
    from stylemc_amd.torch_utils.ops import bias_act
    gen = torch.Generator().manual_seed(0)
    for act in ("tanh", "sigmoid", "elu", "selu", "softplus", "swish"):
        x0 = torch.randn(2, 3, 5, 7, generator=gen)
        b0 = torch.randn(3, generator=gen)
        outs = []
        for dev, fn in ((DEV, bias_act.bias_act), ("cpu", O.bias_act)):
            x = x0.to(dev).requires_grad_(True)
            b = b0.to(dev).requires_grad_(True)
            y = fn(x, b, act=act)
            (gx,) = torch.autograd.grad(y.square().sum(), x, create_graph=True)
            (ggx,) = torch.autograd.grad(gx.sum(), x)
            outs.append((y, gx, ggx))
        for a, r, nm in zip(outs[0], outs[1], ("y", "dx", "ddx")):
            close(a, r, 2e-5, f"{act} {nm}")
    x = torch.randn(6, 9, generator=gen)
    b = torch.randn(6, generator=gen)
    close(bias_act.bias_act(x.to(DEV), b.to(DEV), dim=0, act="lrelu", alpha=0.1, gain=3.0, clamp=2.0),
          O.bias_act(x, b, dim=0, act="lrelu", alpha=0.1, gain=3.0, clamp=2.0), 1e-6, "dim0")
    # odd sizes exercise the scalar path
    x = torch.randn(3, 5, 3, 3, generator=gen)
    close(bias_act.bias_act(x.to(DEV), b[:5].to(DEV), act="lrelu", clamp=0.5),
          O.bias_act(x, b[:5], act="lrelu", clamp=0.5), 1e-6, "odd")


UFD = ["blur_conv0", "up2_img", "down2_adj", "blur_adj", "rect_up2_down1", "crop_neg_pad", "odd_filter",
       "sep_filter8", "up4_down3", "single_pixel"]


@pytest.mark.parametrize("case", UFD)
def test_upfirdn2d_golden(golden, case):
    from stylemc_amd.torch_utils.ops import upfirdn2d
    g = golden("ops_upfirdn2d.npz")
    p = lambda k: g[f"{case}/{k}"]
    x = t(p("x"), DEV).requires_grad_(True)
    y = upfirdn2d.upfirdn2d(x, t(p("f"), DEV), up=[int(v) for v in p("up")], down=[int(v) for v in p("down")],
                            padding=[int(v) for v in p("pad")], flip_filter=bool(p("flip")), gain=float(p("gain")))
    close(y, p("y"), 1e-5, f"{case} y")
    (dx,) = torch.autograd.grad(y, x, t(p("dy"), DEV))
    close(dx, p("dx"), 1e-5, f"{case} dx")


@pytest.mark.parametrize("shape,up,down,pad,flip", [
    ((2, 3, 256, 256), 2, 1, [2, 1, 2, 1], False),     # img upsample at 512
    ((1, 64, 129, 129), 1, 1, [1, 1, 1, 1], False),    # conv0 blur
    ((1, 64, 128, 128), 1, 1, [2, 2, 2, 2], True),     # blur adjoint
    ((2, 3, 512, 512), 1, 2, [1, 2, 1, 2], True),      # upsample adjoint
    ((1, 2, 37, 300), 3, 2, [5, -2, 0, 3], False),     # ragged generic
])
def test_upfirdn2d_vs_oracle_large(shape, up, down, pad, flip):
    from oracle import ops as O
    from stylemc_amd.torch_utils.ops import upfirdn2d
    gen = torch.Generator().manual_seed(1)
    x = torch.randn(shape, generator=gen)
    f = O.setup_filter([1, 3, 3, 1])
    ref = O.upfirdn2d(x, f, up=up, down=down, padding=pad, flip_filter=flip, gain=4)
    out = upfirdn2d.upfirdn2d(x.to(DEV), f.to(DEV), up=up, down=down, padding=pad, flip_filter=flip, gain=4)
    close(out, ref, 1e-5, "upfirdn2d large")


def _pair_layers(cin, cout, res, up, clamp, seed=0, kind="conv"):
    from oracle import networks as ON
    from stylemc_amd import networks as PN
    if kind == "conv":
        o = ON.SynthesisLayer(cin, cout, 512, res, up=up, conv_clamp=clamp)
        p = PN.SynthesisLayer(cin, cout, 512, res, up=up, conv_clamp=clamp)
    else:
        o = ON.ToRGBLayer(cin, 3, 512, conv_clamp=clamp)
        p = PN.ToRGBLayer(cin, 3, 512, conv_clamp=clamp)
    gen = torch.Generator().manual_seed(seed)
    sd = {}
    for k, v in o.state_dict().items():
        if k.endswith("resample_filter"):
            sd[k] = v
        elif k.endswith("noise_strength") or k.endswith("bias"):
            sd[k] = torch.randn(v.shape, generator=gen) * 0.3
        else:
            sd[k] = torch.randn(v.shape, generator=gen)
    o.load_state_dict(sd)
    p.load_state_dict(sd)
    o.affine = torch.nn.Identity()
    p.affine = torch.nn.Identity()
    return o.eval(), p.to(DEV).eval()


def kink_footprint(y_gpu, y_ref, up, clamp=None):
    """Input positions [n, h, w] whose gradient may legitimately differ between the two fp32 evaluations: an
    output element whose pre-activation sits within rounding of an activation kink (lrelu at 0, the clamp)
    can take the other branch on one side -- visible as a different sign, or a different clamped state, of
    the two outputs -- and that one flipped derivative reaches every input channel at every position of the
    conv adjoint's footprint (3x3, or for up = 2 the 4x4 blur adjoint then the stride-2 3x3 gather: dilate 2)."""
    a = y_gpu.detach().double().cpu()
    b = y_ref.detach().double().cpu()
    amb = (a > 0) != (b > 0)
    if clamp is not None:
        amb |= (a.abs() >= clamp) != (b.abs() >= clamp)
    namb = int(amb.sum())
    assert namb <= max(2, amb.numel() // 1000), f"{namb} outputs on different sides of a kink"
    amb = amb.any(dim=1).double()[:, None]
    if up == 2:
        amb = F_pool(amb, 2)
    k = 5 if up == 2 else 3
    return torch.nn.functional.max_pool2d(amb, k, stride=1, padding=k // 2)[:, 0] > 0


def F_pool(t, k):
    return torch.nn.functional.max_pool2d(t, k, stride=k)


def close_grad_outside(a, b, foot, tol, what=""):
    """close_grad for an input gradient, excluding the kink footprint (kink_footprint, which bounds the number
    of disagreeing outputs)."""
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    keep = ~foot[:, None].expand_as(b)
    scale = max(b.abs().max().item(), 1e-12)
    err = (a - b).abs()[keep]
    assert err.numel() == 0 or err.max().item() <= tol * scale, f"{what}: max err {err.max():.3e} > {tol:.1e} * {scale:.3e}"
    rel = ((a - b)[keep].norm() / max(b[keep].norm().item(), 1e-30)).item()
    assert rel <= tol, f"{what}: relative norm error {rel:.3e} > {tol:.1e}"


@pytest.mark.parametrize("cin,cout,res,up,n", [
    (32, 32, 16, 1, 2), (64, 32, 32, 2, 2), (512, 512, 4, 1, 3), (512, 512, 8, 2, 2), (128, 64, 64, 1, 1),
    (256, 128, 32, 2, 1), (512, 256, 16, 2, 4),
])
@pytest.mark.parametrize("noise_mode", ["const", "none"])
def test_synthesis_layer_vs_oracle(cin, cout, res, up, n, noise_mode):
    o, p = _pair_layers(cin, cout, res, up, clamp=1.0 if cin == 32 else 256.0)
    gen = torch.Generator().manual_seed(3)
    x = torch.randn(n, cin, res // up, res // up, generator=gen)
    s = torch.randn(n, cin, generator=gen) * 0.5 + 1
    cot = torch.randn(n, cout, res, res, generator=gen)
    xr, sr = x.clone().requires_grad_(True), s.clone().requires_grad_(True)
    yr = o(xr, sr, noise_mode=noise_mode, fused_modconv=True)
    dxr, dsr = torch.autograd.grad((yr * cot).sum(), [xr, sr])
    xg, sg = x.to(DEV).requires_grad_(True), s.to(DEV).requires_grad_(True)
    yg = p(xg, sg, noise_mode=noise_mode)
    dxg, dsg = torch.autograd.grad((yg * cot.to(DEV)).sum(), [xg, sg])
    close(yg, yr, 2e-5, "y")
    foot = kink_footprint(yg, yr, up, o.conv_clamp)
    close_grad_outside(dxg, dxr, foot, 1e-4, "dx")
    close_grad(dsg, dsr, 1e-4 if not foot.any() else 2e-3, "ds", max_flips=0)


def test_synthesis_layer_grad_subsets():
    """needs_input_grad pruning: styles-only and x-only backward give the same numbers."""
    o, p = _pair_layers(64, 64, 16, 2, clamp=256.0)
    gen = torch.Generator().manual_seed(4)
    x = torch.randn(2, 64, 8, 8, generator=gen).to(DEV)
    s = (torch.randn(2, 64, generator=gen) * 0.5 + 1).to(DEV)
    cot = torch.randn(2, 64, 16, 16, generator=gen).to(DEV)
    xa, sa = x.clone().requires_grad_(True), s.clone().requires_grad_(True)
    dxa, dsa = torch.autograd.grad((p(xa, sa, noise_mode="const") * cot).sum(), [xa, sa])
    sb = s.clone().requires_grad_(True)
    (dsb,) = torch.autograd.grad((p(x, sb, noise_mode="const") * cot).sum(), [sb])
    xc = x.clone().requires_grad_(True)
    (dxc,) = torch.autograd.grad((p(xc, s, noise_mode="const") * cot).sum(), [xc])
    close(dsb, dsa, 1e-6, "ds only")
    close(dxc, dxa, 1e-6, "dx only")


def _both_forms(monkeypatch, run, what):
    """run() -> [(gpu result, fp64 reference), ...] once with split-bf16 products (modconv.X3) and once with the
    exact-fp32 MFMA.  Exact fp32: within 2e-5 of the max vs fp64 (no activation, so no kinks).  Split-bf16: within
    2x the exact-fp32 kernel's own error on the same inputs, in max and in relative norm (the
    three dropped cross terms of a split product are <= 2^-23 |a b|, one fp32 rounding)."""
    from stylemc_amd import modconv
    errs = {}
    for form in (False, True):
        monkeypatch.setattr(modconv, "X3", form)
        out = []
        for got, ref in run(form):
            got = got.detach().double().cpu()
            scale = max(ref.abs().max().item(), 1e-12)
            out.append(((got - ref).abs().max().item() / scale, ((got - ref).norm() / ref.norm()).item()))
        errs[form] = out
    for k, ((f_max, f_norm), (x_max, x_norm)) in enumerate(zip(errs[False], errs[True])):
        assert f_max <= 2e-5, f"{what}[{k}] exact fp32: max err {f_max:.3e}"
        assert x_max <= 2 * f_max, f"{what}[{k}] x3 max err {x_max:.3e} > 2 x fp32 {f_max:.3e}"
        assert x_norm <= 2 * f_norm, f"{what}[{k}] x3 norm err {x_norm:.3e} > 2 x fp32 {f_norm:.3e}"


@pytest.mark.parametrize("n,cin,cout,r", [(2, 32, 32, 256), (4, 64, 32, 128), (1, 32, 32, 1024), (2, 64, 64, 128),
                                           (1, 96, 64, 256), (2, 64, 64, 256), (1, 128, 128, 128), (1, 256, 256, 128),
                                           (2, 512, 512, 16), (4, 512, 512, 8), (3, 128, 64, 24)])
def test_conv_gemm_same3x3_vs_conv2d(n, cin, cout, r, monkeypatch):
    """3x3 'same' convs (conv1 forward with per-sample style-scaled weights, and its data gradient with the
    shared flipped weights) against an fp64 CPU convolution.  Exact-fp32 MFMA: 32 / 64 output channels with
    W % 256 == 0 run the row-halo kernel (conv_row_kernel, both tile widths), the other shapes the tap-major LDS-DMA
    kernel; split-bf16: every shape the LDS-DMA tiles with split products (per-sample split weights in the forward,
    split-K at 8 and 16 px)."""
    import torch.nn.functional as F
    from stylemc_amd import _hip, modconv
    gen = torch.Generator().manual_seed(11)
    W = torch.randn(cout, cin, 3, 3, generator=gen)
    x = torch.randn(n, cin, r, r, generator=gen)
    s = torch.randn(n, cin, generator=gen) * 0.5 + 1
    g = torch.randn(n, cout, r, r, generator=gen)
    ref = F.conv2d((x * s[:, :, None, None]).double(), W.double(), padding=1)
    refb = F.conv_transpose2d(g.double(), W.double(), padding=1)

    def run(form):
        P = modconv.PackedConv(W.to(DEV), 1)
        ph, nph, _, _ = P.fwd_phases(r, r)
        y = torch.empty(n, cout, r, r, device=DEV)
        modconv.gemm(x.to(DEV), y, ph, nph, cin, cout, s=s.to(DEV), epi=modconv._epilogue(_hip.EPI_STORE))
        phb, nphb = P.bwd_phases(r, r)
        dx = torch.empty(n, cin, r, r, device=DEV)
        modconv.gemm(g.to(DEV), dx, phb, nphb, cout, cin, epi=modconv._epilogue(_hip.EPI_STORE))
        assert (P.x3_fwd is not None) == form
        return [(y, ref), (dx, refb)]

    _both_forms(monkeypatch, run, "3x3 fwd / data grad")


@pytest.mark.parametrize("n,cin,cout,h", [(2, 64, 32, 64), (1, 32, 32, 128), (2, 512, 512, 4), (3, 256, 128, 16),
                                           (1, 128, 64, 64)])
def test_conv_gemm_stride2_gather_vs_conv2d(n, cin, cout, h, monkeypatch):
    """The up = 2 layers' data gradient through the transposed conv: the stride-2 3x3 gather over dT (2h + 1 rows,
    a padded pitch) against an fp64 conv2d(stride 2) of the same dT, both product forms (_both_forms)."""
    import torch.nn.functional as F
    from stylemc_amd import _hip, modconv
    gen = torch.Generator().manual_seed(17)
    W = torch.randn(cout, cin, 3, 3, generator=gen)
    th = 2 * h + 1
    g = torch.randn(n, cout, th, th, generator=gen)
    ref = F.conv2d(g.double(), W.transpose(0, 1).double(), stride=2)

    def run(form):
        P = modconv.PackedConv(W.to(DEV), 2)
        phb, nphb = P.bwd_phases(h, h)
        dx = torch.empty(n, cin, h, h, device=DEV)
        modconv.gemm(g.to(DEV), dx, phb, nphb, cout, cin, epi=modconv._epilogue(_hip.EPI_STORE))
        assert ref.shape == dx.shape, (ref.shape, dx.shape)
        assert (P.x3_bwd is not None) == form
        return [(dx, ref)]

    _both_forms(monkeypatch, run, "stride-2 gather")


@pytest.mark.parametrize("n,cin,cout,h", [(2, 64, 32, 64), (1, 128, 64, 128), (2, 512, 512, 4), (3, 256, 128, 16),
                                           (1, 512, 256, 32), (2, 32, 32, 33), (4, 512, 512, 8)])
def test_conv_gemm_transposed_vs_conv_transpose2d(n, cin, cout, h, monkeypatch):
    """The up = 2 layers' stride-2 transposed 3x3 conv (conv2d_resample.py:125-138 before the blur) as the
    phase-fused LDS-DMA kernel: per-sample style-scaled weights with tiles restarted per image ((h+1)^2 not a
    tile multiple), a prescaled input at the low resolutions, split-K over channel chunks; vs fp64
    conv_transpose2d, both product forms (_both_forms)."""
    import torch.nn.functional as F
    from stylemc_amd import _hip, modconv
    gen = torch.Generator().manual_seed(13)
    W = torch.randn(cout, cin, 3, 3, generator=gen)
    x = torch.randn(n, cin, h, h, generator=gen)
    s = torch.randn(n, cin, generator=gen) * 0.5 + 1
    ref = F.conv_transpose2d((x * s[:, :, None, None]).double(), W.transpose(0, 1).double(), stride=2)

    def run(form):
        P = modconv.PackedConv(W.to(DEV), 2)
        ph, nph, th, tw = P.fwd_phases(h, h)
        t = torch.empty(n, cout, th, tw, device=DEV)
        modconv.gemm(x.to(DEV), t, ph, nph, cin, cout, s=s.to(DEV), epi=modconv._epilogue(_hip.EPI_STORE))
        assert all((w is not None) == form for w in P.x3_phases)
        return [(t, ref)]

    _both_forms(monkeypatch, run, "transposed conv")


@pytest.mark.parametrize("kind", ["transposed", "stride2"])
def test_conv_gemm_x3_wide_tile(kind, monkeypatch):
    """The split-bf16 wide tile (256 output channels x 128 positions, conv_gemm_x3_kernel AS: A fragments streamed per
    output block, the epilogue in two halves) where its grid fills the chip unsplit -- one image planned as 16
    (_hip.plan_batch), the r = 128 conv0 forward / r = 256 data-gradient shapes of the 4-image step: vs fp64, both
    product forms (_both_forms), and the library reports the wide launch (smc_conv_gemm_last_x3 == 2)."""
    import torch.nn.functional as F
    from stylemc_amd import _hip, modconv
    gen = torch.Generator().manual_seed(23)
    lib = _hip.load()
    if kind == "transposed":
        cin, cout, h = 512, 256, 32
        W = torch.randn(cout, cin, 3, 3, generator=gen)
        x = torch.randn(1, cin, h, h, generator=gen)
        s = torch.randn(1, cin, generator=gen) * 0.5 + 1
        ref = F.conv_transpose2d((x * s[:, :, None, None]).double(), W.transpose(0, 1).double(), stride=2)
    else:
        cin, cout, h = 256, 128, 64   # the forward's channels; the data gradient has cin = 256 outputs
        W = torch.randn(cout, cin, 3, 3, generator=gen)
        g = torch.randn(1, cout, 2 * h + 1, 2 * h + 1, generator=gen)
        ref = F.conv2d(g.double(), W.transpose(0, 1).double(), stride=2)

    def run(form):
        P = modconv.PackedConv(W.to(DEV), 2)
        with _hip.plan_batch(16, 1):
            if kind == "transposed":
                ph, nph, th, tw = P.fwd_phases(h, h)
                out = torch.empty(1, cout, th, tw, device=DEV)
                modconv.gemm(x.to(DEV), out, ph, nph, cin, cout, s=s.to(DEV), epi=modconv._epilogue(_hip.EPI_STORE))
            else:
                phb, nphb = P.bwd_phases(h, h)
                out = torch.empty(1, cin, h, h, device=DEV)
                modconv.gemm(g.to(DEV), out, phb, nphb, cout, cin, epi=modconv._epilogue(_hip.EPI_STORE))
            assert lib.smc_conv_gemm_last_x3() == (2 if form else 0)
        return [(out, ref)]

    _both_forms(monkeypatch, run, f"wide tile {kind}")


def _misaligned(t):
    """A copy of `t` whose data pointer is 4 B past a 16-B boundary (forces the scalar-load kernels)."""
    buf = torch.empty(t.numel() + 1, device=t.device, dtype=t.dtype)
    v = buf[1:].view(t.shape)
    v.copy_(t)
    assert v.data_ptr() % 16 == 4
    return v


@pytest.mark.parametrize("n,c,h", [(2, 8, 64), (1, 4, 37), (2, 3, 256), (1, 2, 100)])
def test_blur_act_load_paths(n, c, h):
    """conv0's fused FIR + modconv epilogue (smc_modconv_blur_act_f32) and its backward: the 16-B load kernels
    (16-B aligned buffers; any T row pitch, incl. the transposed conv's odd 2h + 1 and an explicit padded pitch)
    against the scalar-load kernels (a misaligned copy of the same buffers) -- the same FIR arithmetic, so y, u and
    dT must agree bit for bit (dd: block sums in a different atomic order, 4e-6 of the max) -- and U against fp64 torch."""
    import ctypes
    import torch.nn.functional as F
    from stylemc_amd import _hip, modconv
    gen = torch.Generator().manual_seed(21)
    th, r = 2 * h + 1, 2 * h
    f1 = torch.tensor([1.0, 3.0, 3.0, 1.0])
    f = (f1[:, None] * f1[None, :] / 64.0).to(DEV)
    T = torch.randn(n, c, th, th, generator=gen).to(DEV)
    d = (torch.rand(n, c, generator=gen) + 0.5).to(DEV)
    noise = torch.randn(r, r, generator=gen).to(DEV)
    strength = torch.tensor(0.3, device=DEV)
    bias = (torch.randn(c, generator=gen) * 0.1).to(DEV)
    st = _hip.stream()

    def fwd(tbuf, pitch, builtin=False):
        y = torch.empty(n, c, r, r, device=DEV)
        u = torch.empty_like(y)
        epi = modconv._epilogue(_hip.EPI_MODACT, d, noise, 0, strength, bias, "lrelu", 0.2, 2 ** 0.5, 1.0, u)
        _hip.call("smc_modconv_blur_act_f32", tbuf.data_ptr(), 1, 0, y.data_ptr(), n, c, th, th, pitch, r, r,
                  None if builtin else f.data_ptr(), 4, 4, 1, 1, 4.0, 0, ctypes.byref(epi), st)
        return y, u

    y0, u0 = fwd(T, 0)
    Tp = torch.zeros(n, c, th, th + 7, device=DEV)
    Tp[..., :th] = T
    y1, u1 = fwd(Tp, th + 7)
    y2, u2 = fwd(_misaligned(T), 0)
    y3, u3 = fwd(T, 0, builtin=True)               # f = NULL: compile-time [1,3,3,1] taps (16-B kernel)
    y4, u4 = fwd(_misaligned(T), 0, builtin=True)  # ... and the scalar-load kernel's built-in taps
    torch.cuda.synchronize()
    for a, b, what in ((y1, y0, "y pitched"), (u1, u0, "u pitched"), (y2, y0, "y scalar"), (u2, u0, "u scalar"),
                       (y3, y0, "y built-in taps"), (u3, u0, "u built-in taps"), (y4, y0, "y scalar built-in"),
                       (u4, u0, "u scalar built-in")):
        assert torch.equal(a, b), what
    ref = F.conv2d(F.pad(T.double().cpu(), (1, 1, 1, 1)).view(n * c, 1, th + 2, th + 2),
                   (4.0 * f.double().cpu().flip(0, 1))[None, None]).view(n, c, r, r)
    close(u0, ref, 2e-6, "U vs fp64")

    g = torch.randn(n, c, r, r, generator=gen).to(DEV)

    def bwd(gb, ub):
        dt = torch.full((n, c, th, th), float("nan"), device=DEV)
        dd = torch.zeros(n, c, device=DEV)
        epi = modconv._epilogue(_hip.EPI_MODACT, d, noise, 0, strength, bias, "lrelu", 0.2, 2 ** 0.5, 1.0)
        ws = _dd_ws("smc_modconv_blur_act_bwd_workspace_size", n, c, r, r, th, th)
        _hip.call("smc_modconv_blur_act_bwd_f32", gb.data_ptr(), ub.data_ptr(), dt.data_ptr(), dd.data_ptr(), n, c,
                  r, r, th, th, 0, f.data_ptr(), 4, 4, 2, 2, 4.0, 1, ctypes.byref(epi), _hip.ptr(ws), _nb(ws), st)
        return dt, dd

    dt0, dd0 = bwd(g, u0)
    dt1, dd1 = bwd(_misaligned(g), _misaligned(u0))
    _, dd0b = bwd(g, u0)

    def bwd_from_y(gb, yb, builtin=False):   # grad_from_y: the saved forward output instead of u, no dd
        dt = torch.full((n, c, th, th), float("nan"), device=DEV)
        epi = modconv._epilogue(_hip.EPI_MODACT, d, noise, 0, strength, bias, "lrelu", 0.2, 2 ** 0.5, 1.0)
        epi.grad_from_y = 1
        _hip.call("smc_modconv_blur_act_bwd_f32", gb.data_ptr(), yb.data_ptr(), dt.data_ptr(), None, n, c,
                  r, r, th, th, 0, None if builtin else f.data_ptr(), 4, 4, 2, 2, 4.0, 1, ctypes.byref(epi), None, 0,
                  st)
        return dt

    dt2 = bwd_from_y(g, y0)
    dt3 = bwd_from_y(_misaligned(g), _misaligned(y0))
    dt4 = bwd_from_y(g, y0, builtin=True)              # built-in [1,3,3,1] taps (16-B kernel)
    dt5 = bwd_from_y(_misaligned(g), _misaligned(y0), builtin=True)
    assert torch.equal(dt4, dt2) and torch.equal(dt5, dt2), "dT built-in taps vs the filter tensor"
    torch.cuda.synchronize()
    assert torch.isfinite(dt0).all()
    assert torch.equal(dt0, dt1), "dT scalar vs 16-B loads"
    # dd: planes with more than two dd-owning tiles store per-tile partials that a fixed-order pass sums, so the result
    # is bit-reproducible run to run; the two load paths order a tile's own sum differently (fp32 rounding apart)
    assert torch.equal(dd0, dd0b), "dd run to run"
    close(dd1, dd0, 1e-5, "dd scalar vs 16-B loads")
    close(dd0, _dd_ref(g, u0, d, noise, strength, bias), 1e-5, "dd vs fp64")
    # y = epi_y(u) bit for bit, so the mask and dT are identical
    assert torch.equal(dt2, dt0), "dT from y vs from u"
    assert torch.equal(dt3, dt0), "dT from y, scalar loads"


def _dd_ws(query, *dims):
    """The caller-owned dd-partials workspace the epilogue backward kernels ask for (None when they need none)."""
    from stylemc_amd import _hip
    nbytes = getattr(_hip.load(), query)(*dims)
    return torch.empty(nbytes // 4, device=DEV) if nbytes > 0 else None


def _nb(t):
    return 0 if t is None else 4 * t.numel()


def _dd_ref(g, u, d, noise, strength, bias, alpha=0.2, gain=2 ** 0.5, clamp=1.0):
    """dd[n, o] = sum_hw dz * u in fp64: the gradient of <g, y(u d + noise strength + bias)> w.r.t. d."""
    u64 = u.double().cpu()
    dv = d.double().cpu().clone().requires_grad_(True)
    z = u64 * dv[:, :, None, None] + noise.double().cpu() * strength.double().cpu() + bias.double().cpu()[None, :, None, None]
    y = (torch.nn.functional.leaky_relu(z, alpha) * gain).clamp(-clamp, clamp)
    (dd,) = torch.autograd.grad(y, dv, g.double().cpu())
    return dd


@pytest.mark.parametrize("hw", [(256, 256), (96, 100)])
def test_act_bwd_dd_deterministic(hw):
    """dd of conv1's epilogue backward on planes that span more than two workgroups: per-workgroup partials summed
    per plane in a fixed order -- bit-equal run to run and against the fp64 reference (1e-5 of the max)."""
    import ctypes
    from stylemc_amd import _hip, modconv
    gen = torch.Generator().manual_seed(23)
    n, c = 2, 16
    h, w = hw
    u = torch.randn(n, c, h, w, generator=gen).to(DEV)
    g = torch.randn(n, c, h, w, generator=gen).to(DEV)
    d = (torch.rand(n, c, generator=gen) + 0.5).to(DEV)
    noise = torch.randn(h, w, generator=gen).to(DEV)
    strength = torch.tensor(0.3, device=DEV)
    bias = (torch.randn(c, generator=gen) * 0.1).to(DEV)
    epi = modconv._epilogue(_hip.EPI_MODACT, d, noise, 0, strength, bias, "lrelu", 0.2, 2 ** 0.5, 1.0)
    outs = []
    for _ in range(3):
        du, dd = torch.empty_like(u), torch.zeros(n, c, device=DEV)
        ws = _dd_ws("smc_modconv_act_bwd_workspace_size", n, c, h, w)
        _hip.call("smc_modconv_act_bwd_f32", g.data_ptr(), u.data_ptr(), du.data_ptr(), dd.data_ptr(), n, c, h, w,
                  ctypes.byref(epi), _hip.ptr(ws), _nb(ws), _hip.stream())
        outs.append((du, dd))
    du_n, dd_none = torch.empty_like(u), None
    _hip.call("smc_modconv_act_bwd_f32", g.data_ptr(), u.data_ptr(), du_n.data_ptr(), None, n, c, h, w,
              ctypes.byref(epi), None, 0, _hip.stream())
    torch.cuda.synchronize()
    for du, dd in outs[1:]:
        assert torch.equal(dd, outs[0][1]) and torch.equal(du, outs[0][0])
    assert torch.equal(du_n, outs[0][0])
    close(outs[0][1], _dd_ref(g, u, d, noise, strength, bias), 1e-5, "dd vs fp64")


@pytest.mark.parametrize("uhw", [(128, 128), (64, 192)])
def test_blur_act_bwd_dd_two_level(uhw):
    """dd of conv0's fused epilogue + FIR backward on planes with more than two dd-owning tiles (per-tile partials,
    then a fixed-order per-plane sum): bit-equal run to run, dT equal to the dd-free call, dd within 1e-5 of the fp64
    reference."""
    import ctypes
    from stylemc_amd import _hip, modconv
    gen = torch.Generator().manual_seed(29)
    n, c = 2, 8
    uh, uw = uhw
    th, tw = uh + 1, uw + 1
    pitch = (tw + 3) // 4 * 4
    u = torch.randn(n, c, uh, uw, generator=gen).to(DEV)
    g = torch.randn(n, c, uh, uw, generator=gen).to(DEV)
    d = (torch.rand(n, c, generator=gen) + 0.5).to(DEV)
    noise = torch.randn(uh, uw, generator=gen).to(DEV)
    strength = torch.tensor(0.3, device=DEV)
    bias = (torch.randn(c, generator=gen) * 0.1).to(DEV)
    f1 = torch.tensor([1., 3., 3., 1.], device=DEV)
    f = (f1[:, None] * f1[None, :] / 64.0).contiguous()
    epi = modconv._epilogue(_hip.EPI_MODACT, d, noise, 0, strength, bias, "lrelu", 0.2, 2 ** 0.5, 1.0)

    def run(with_dd):
        dt = torch.zeros(n, c, th, pitch, device=DEV)
        dd = torch.zeros(n, c, device=DEV) if with_dd else None
        ws = _dd_ws("smc_modconv_blur_act_bwd_workspace_size", n, c, uh, uw, th, tw) if with_dd else None
        _hip.call("smc_modconv_blur_act_bwd_f32", g.data_ptr(), u.data_ptr(), dt.data_ptr(), _hip.ptr(dd), n, c, uh,
                  uw, th, tw, pitch, f.data_ptr(), 4, 4, 2, 2, 4.0, 1, ctypes.byref(epi), _hip.ptr(ws), _nb(ws),
                  _hip.stream())
        return dt, dd

    outs = [run(True) for _ in range(3)]
    dt_n, _ = run(False)
    torch.cuda.synchronize()
    for dt, dd in outs[1:]:
        assert torch.equal(dd, outs[0][1]) and torch.equal(dt, outs[0][0])
    assert torch.equal(dt_n, outs[0][0])
    close(outs[0][1], _dd_ref(g, u, d, noise, strength, bias), 1e-5, "dd vs fp64")


@pytest.mark.parametrize("hw", [(64, 64), (7, 9)])
def test_act_bwd_from_y(hw):
    """conv1's epilogue backward (smc_modconv_act_bwd_f32) from the saved output y (grad_from_y: layers whose styles
    need no gradient keep no u) equals the u path bit for bit (float4 and scalar kernels)."""
    import ctypes
    from stylemc_amd import _hip, modconv
    gen = torch.Generator().manual_seed(22)
    n, c = 2, 8
    h, w = hw
    u = torch.randn(n, c, h, w, generator=gen).to(DEV)
    g = torch.randn(n, c, h, w, generator=gen).to(DEV)
    d = (torch.rand(n, c, generator=gen) + 0.5).to(DEV)
    noise = torch.randn(h, w, generator=gen).to(DEV)
    strength = torch.tensor(0.3, device=DEV)
    bias = (torch.randn(c, generator=gen) * 0.1).to(DEV)
    st = _hip.stream()
    y = torch.empty_like(u)
    epi = modconv._epilogue(_hip.EPI_MODACT, d, noise, 0, strength, bias, "lrelu", 0.2, 2 ** 0.5, 1.0)
    _hip.call("smc_modconv_epilogue_f32", u.data_ptr(), 1, 0, y.data_ptr(), n, c, h, w, ctypes.byref(epi), st)
    du0, du1 = torch.empty_like(u), torch.empty_like(u)
    dd = torch.zeros(n, c, device=DEV)
    ws = _dd_ws("smc_modconv_act_bwd_workspace_size", n, c, h, w)
    _hip.call("smc_modconv_act_bwd_f32", g.data_ptr(), u.data_ptr(), du0.data_ptr(), dd.data_ptr(), n, c, h, w,
              ctypes.byref(epi), _hip.ptr(ws), _nb(ws), st)
    epi.grad_from_y = 1
    _hip.call("smc_modconv_act_bwd_f32", g.data_ptr(), y.data_ptr(), du1.data_ptr(), None, n, c, h, w,
              ctypes.byref(epi), None, 0, st)
    torch.cuda.synchronize()
    assert torch.equal(du0, du1)
    with pytest.raises(RuntimeError):   # dd needs u
        _hip.call("smc_modconv_act_bwd_f32", g.data_ptr(), y.data_ptr(), du1.data_ptr(), dd.data_ptr(), n, c, h, w,
                  ctypes.byref(epi), _hip.ptr(ws), _nb(ws), st)


def test_conv_gemm_2gib_input_fallback():
    """An input of >= 2 GiB (batch 16 of the r = 1024 conv1: 2.1 GB) exceeds the 32-bit buffer offsets of the
    LDS-DMA / row-halo kernels and runs the register-staged kernel with 64-bit addressing: it must equal the
    same conv computed in two halves of the batch (each < 2 GiB, the fast kernels), to fp32 summation order."""
    from stylemc_amd import _hip, modconv
    gen = torch.Generator().manual_seed(12)
    n, cin, cout, r = 16, 32, 32, 1024
    assert n * cin * r * r * 4 >= 2 ** 31
    W = torch.randn(cout, cin, 3, 3, generator=gen).to(DEV)
    P = modconv.PackedConv(W, 1)
    x = torch.randn(n, cin, r, r, device=DEV)
    s = torch.rand(n, cin, device=DEV) + 0.5
    ph, nph, _, _ = P.fwd_phases(r, r)
    y = torch.empty(n, cout, r, r, device=DEV)
    modconv.gemm(x, y, ph, nph, cin, cout, s=s, epi=modconv._epilogue(_hip.EPI_STORE))
    y2 = torch.empty_like(y)
    h = n // 2
    for sl in (slice(0, h), slice(h, n)):
        part = torch.empty(h, cout, r, r, device=DEV)
        modconv.gemm(x[sl].contiguous(), part, ph, nph, cin, cout, s=s[sl].contiguous(),
                     epi=modconv._epilogue(_hip.EPI_STORE))
        y2[sl] = part
    err = ((y - y2).abs().max() / y2.abs().max()).item()
    assert err <= 2e-6, err
    del x, y, y2
    torch.cuda.empty_cache()


@pytest.mark.parametrize("cin,res,n,clamp", [(512, 4, 2, 256.0), (64, 64, 3, 0.3), (32, 128, 1, None), (128, 9, 2, 1.0)])
def test_torgb_vs_oracle(cin, res, n, clamp):
    o, p = _pair_layers(cin, 3, res, 1, clamp=clamp, kind="rgb")
    gen = torch.Generator().manual_seed(5)
    x = torch.randn(n, cin, res, res, generator=gen)
    s = torch.randn(n, cin, generator=gen) * 0.5 + 1
    cot = torch.randn(n, 3, res, res, generator=gen)
    xr, sr = x.clone().requires_grad_(True), s.clone().requires_grad_(True)
    yr = o(xr, sr)
    dxr, dsr = torch.autograd.grad((yr * cot).sum(), [xr, sr])
    xg, sg = x.to(DEV).requires_grad_(True), s.to(DEV).requires_grad_(True)
    yg = p(xg, sg)
    dxg, dsg = torch.autograd.grad((yg * cot.to(DEV)).sum(), [xg, sg])
    close(yg, yr, 2e-5, "y")
    close(dxg, dxr, 2e-5, "dx")
    close(dsg, dsr, 1e-4, "ds")


def _product_G(res, cbase, clamp, seed=7):
    from stylemc_amd import networks, synthetic
    cfg = synthetic.generator_config(resolution=res, channel_base=cbase, conv_clamp=clamp)
    return networks.build_generator(cfg, synthetic.generator_state_dict(cfg, seed=seed), device=DEV)


@pytest.mark.parametrize("tag", ["r32", "r16_clamp"])
def test_synthesis_tiny_golden(golden, tag):
    """Whole S-space synthesis fwd + style gradients vs vectors from the reference's own driver."""
    from stylemc_amd import utils
    g = golden("synthesis_tiny.npz")
    res, cbase, n, until_k = [int(v) for v in g[f"{tag}/meta"]]
    G = _product_G(res, cbase, float(g[f"{tag}/clamp"]))
    shapes = utils.get_temp_shapes(G)
    styles = t(g[f"{tag}/styles"], DEV).requires_grad_(True)
    xs, img = utils.generate_image(G, until_k, styles, shapes, "const")
    for k, xk in enumerate(xs):
        close(xk, g[f"{tag}/xs{k}"], 1e-4, f"xs{k}")
    close(img, g[f"{tag}/img"], 1e-4, "img")
    (ds,) = torch.autograd.grad((img * t(g[f"{tag}/cot"], DEV)).sum(), styles)
    close(ds, g[f"{tag}/dstyles"], 1e-3, "dstyles")


def test_synthesis_1024_vs_oracle():
    """FFHQ-1024 config-f geometry, N=1: full forward image + direction-row gradients vs the CPU oracle."""
    from oracle import networks as ON
    from oracle import synthesis as OS
    from stylemc_amd import synthetic, utils
    cfg = synthetic.generator_config(resolution=1024)
    sd = synthetic.generator_state_dict(cfg, seed=0)
    G = _product_G(1024, 32768, 256.0, seed=0)
    Go = torch.nn.Module()
    Go.synthesis = ON.SynthesisNetwork(512, 1024, 3, channel_base=32768, conv_clamp=256.0)
    Go.synthesis.load_state_dict({k[10:]: v for k, v in sd.items() if k.startswith("synthesis.")}, strict=False)
    Go.eval().requires_grad_(False)
    shapes_p, shapes_o = utils.get_temp_shapes(G), OS.get_temp_shapes(Go)
    assert shapes_p == shapes_o
    styles = synthetic.synthetic_styles(1, seed=0)
    gen = torch.Generator().manual_seed(2)
    cot = torch.randn(1, 3, 1024, 1024, generator=gen)
    so = styles.clone().requires_grad_(True)
    _, img_o = OS.generate_image(Go, 8, so, shapes_o, "const")
    (ds_o,) = torch.autograd.grad((img_o * cot).sum(), so)
    sp = styles.to(DEV).requires_grad_(True)
    _, img_p = utils.generate_image(G, 8, sp, shapes_p, "const")
    (ds_p,) = torch.autograd.grad((img_p * cot.to(DEV)).sum(), sp)
    close(img_p, img_o, 1e-4, "img 1024")
    T = utils.S_TRAINABLE_SPACE_CHANNELS
    close(ds_p[:, T], ds_o[:, T], 2e-3, "dstyles trainable rows")
    cos = torch.nn.functional.cosine_similarity(ds_p.cpu().double().flatten(), ds_o.double().flatten(), dim=0)
    assert cos > 0.9999, cos


@pytest.mark.parametrize("res,ch,styles_grad", [(128, 64, False), (64, 128, True), (1024, 32, False)])
def test_conv1_torgb_fused_backward(res, ch, styles_grad):
    """SynthesisBlock.conv1_torgb (modconv.ModConvToRGBFn: the block output's two gradients -- this block's ToRGB
    and the next block's conv0 -- summed inside conv1's epilogue backward, smc_torgb_act_bwd_f32) against the
    separate conv1 + ToRGB Functions with autograd's sum: bit-identical where conv1's styles need no gradient
    (the fused kernel), 1e-6 otherwise (the same kernels in another order)."""
    from stylemc_amd import networks
    torch.manual_seed(5)
    blk = networks.SynthesisBlock(ch, ch, 512, res, 3, is_last=False, conv_clamp=256).to(DEV)
    with torch.no_grad():
        for p_ in blk.parameters():
            p_.copy_(torch.randn_like(p_) * (0.3 if p_.ndim <= 1 else 1.0))
    n = 2
    x0 = torch.randn(n, ch, res, res, device=DEV)
    w1 = torch.randn(n, 512, device=DEV)
    wr = torch.randn(n, 512, device=DEV)
    g_next = torch.randn(n, ch, res, res, device=DEV)
    g_rgb = torch.randn(n, 3, res, res, device=DEV)
    outs = []
    for fused in (True, False):
        x = x0.clone().requires_grad_(True)
        w = w1.clone().requires_grad_(styles_grad)
        if fused:
            y, rgb = blk.conv1_torgb(x, w, wr, noise_mode="const")
        else:
            y = blk.conv1(x, w, noise_mode="const")
            rgb = blk.torgb(y, wr)
        loss = (y * g_next).sum() + (rgb * g_rgb).sum()
        grads = torch.autograd.grad(loss, [x, w] if styles_grad else [x])
        outs.append((y.detach(), rgb.detach()) + tuple(grads))
    for a, b, what in zip(outs[0], outs[1], ("y", "rgb", "dx", "dw")):
        if styles_grad and what in ("dx", "dw"):
            close(a, b, 1e-6, what)
        else:
            assert torch.equal(a, b), what
    # the last block: ToRGB is the only consumer of y (no g_next)
    x = x0.clone().requires_grad_(True)
    y, rgb = blk.conv1_torgb(x, w1, wr, noise_mode="const")
    (dxa,) = torch.autograd.grad((rgb * g_rgb).sum(), [x])
    x = x0.clone().requires_grad_(True)
    (dxb,) = torch.autograd.grad((blk.torgb(blk.conv1(x, w1, noise_mode="const"), wr) * g_rgb).sum(), [x])
    assert torch.equal(dxa, dxb), "last block"
