"""Winograd F(4x4, 3x3) conv kernel (csrc/wino4.hip) through the C ABI.

Checked against fp64 conv2d on the same fp32 inputs.  Tolerance: every output's error <= TOL4 x sum_k |w_k x_k| (the
fp64 conv of |W| and |x*s|) and the relative norm error <= REL4.  F(4x4) transforms carry the factors 4, 5, 8 and
1/6, 1/24 (U in fp64, rounded once), so its fp32 error is larger than F(2x2)'s (test_gpu_wino.py: 2e-6 / 1e-6); a
numpy model of the same fp32 arithmetic gives ~1.3e-6 max / ~3e-6 relative norm at cin = 256.
The MODACT epilogue (demod, noise, bias, lrelu, clamp, u store) is compared with the F(2x2) kernel on the same
inputs.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"
TOL4 = 8e-6
REL4 = 1e-5


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from stylemc_amd import build
    build.build(verbose=False)
    torch.backends.cudnn.allow_tf32 = False


def _lib():
    from stylemc_amd import _hip
    return _hip


def _check(got, x64, w64, what):
    ref = F.conv2d(x64, w64, padding=1)
    bound = F.conv2d(x64.abs(), w64.abs(), padding=1)
    err = (got.double().cpu() - ref).abs()
    ratio = (err / (bound + 1e-30)).max().item()
    rel = ((got.double().cpu() - ref).norm() / ref.norm()).item()
    print(f"{what}: max err / sum|w x| {ratio:.3e}, relative norm error {rel:.3e}")
    assert ratio <= TOL4, f"{what}: max err / sum|w x| = {ratio:.3e} > {TOL4:.1e}"
    assert rel <= REL4, f"{what}: relative norm error {rel:.3e}"


SHAPES = [  # n, cin, cout, h, w  (non-square, 512 channels, cin != cout, cin % 8 == 4, several work items per image)
    (2, 32, 64, 64, 64),
    (1, 64, 64, 64, 64),
    (2, 16, 64, 128, 128),
    (1, 64, 128, 256, 128),
    (2, 512, 512, 64, 64),
    (1, 128, 128, 64, 256),
    (1, 12, 64, 32, 64),
    (4, 64, 64, 512, 512),
]


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_wino4_forward_vs_fp64(shape):
    H = _lib()
    n, cin, cout, h, w = shape
    g = torch.Generator().manual_seed(sum(shape))
    x = torch.randn(n, cin, h, w, generator=g)
    s = torch.rand(n, cin, generator=g) + 0.5
    W = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    assert H.load().smc_conv3x3_wino4_supported(n, cin, cout, h, w) == 1
    xd, sd, Wd = x.to(DEV), s.to(DEV), W.to(DEV)
    uw = torch.empty(36 * cin * cout, device=DEV)
    H.call("smc_wino4_weights_f32", Wd.data_ptr(), cout, cin, 0, uw.data_ptr(), H.stream())
    y = torch.full((n, cout, h, w), float("nan"), device=DEV)
    H.call("smc_conv3x3_wino4_f32", xd.data_ptr(), n, cin, h, w, y.data_ptr(), cout, uw.data_ptr(), sd.data_ptr(),
           None, H.stream())
    torch.cuda.synchronize()
    assert torch.isfinite(y).all()
    if n * h * w >= 1 << 20:  # the 512-px case: check the first and last rows of every image (fp64 conv is slow)
        for rows in (slice(0, 64), slice(h - 64, h)):
            xs = x[:, :, max(rows.start - 1, 0):min(rows.stop + 1, h)]
            ref_x = xs.double() * s.double()[:, :, None, None]
            ref = F.conv2d(ref_x, W.double(), padding=1)
            bound = F.conv2d(ref_x.abs(), W.double().abs(), padding=1)
            sl = slice(0, 64) if rows.start == 0 else slice(1, 65)
            ref, bound = ref[:, :, sl], bound[:, :, sl]
            got = y[:, :, rows].cpu().double()
            ratio = ((got - ref).abs() / (bound + 1e-30)).max().item()
            assert ratio <= TOL4, ratio
        return
    _check(y, x.double() * s.double()[:, :, None, None], W.double(), f"fwd {shape}")


@pytest.mark.parametrize("shape", SHAPES[:7], ids=lambda s: "x".join(map(str, s)))
def test_wino4_data_grad_vs_fp64(shape):
    """flip = 1 weights: the conv^T of the 3x3 'same' conv (its data gradient) with cin / cout swapped."""
    H = _lib()
    n, cin, cout, h, w = shape
    g = torch.Generator().manual_seed(7 + sum(shape))
    gy = torch.randn(n, cout, h, w, generator=g)
    W = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    if not H.load().smc_conv3x3_wino4_supported(n, cout, cin, h, w):
        pytest.skip("transposed shape has no F(4x4) kernel")
    Wd = W.to(DEV)
    uw = torch.empty(36 * cin * cout, device=DEV)
    H.call("smc_wino4_weights_f32", Wd.data_ptr(), cout, cin, 1, uw.data_ptr(), H.stream())
    dx = torch.empty(n, cin, h, w, device=DEV)
    gyd = gy.to(DEV)
    H.call("smc_conv3x3_wino4_f32", gyd.data_ptr(), n, cout, h, w, dx.data_ptr(), cin, uw.data_ptr(), None, None,
           H.stream())
    torch.cuda.synchronize()
    Wt = W.double().flip(2, 3).transpose(0, 1).contiguous()
    _check(dx, gy.double(), Wt, f"dgrad {shape}")


def test_wino4_weights_vs_fp64():
    H = _lib()
    cout, cin = 64, 32
    W = torch.randn(cout, cin, 3, 3, generator=torch.Generator().manual_seed(3))
    G = torch.tensor([[1 / 4, 0, 0], [-1 / 6, -1 / 6, -1 / 6], [-1 / 6, 1 / 6, -1 / 6], [1 / 24, 1 / 12, 1 / 6],
                      [1 / 24, -1 / 12, 1 / 6], [0, 0, 1]], dtype=torch.float64)
    for flip in (0, 1):
        g = W.double() if flip == 0 else W.double().flip(2, 3).transpose(0, 1)  # [N][K][3][3]
        U = torch.einsum("ai,nkij,bj->knba", G, g, G)     # [K][N][b][a]: xi = 6 b + a
        ref = U.reshape(U.shape[0], U.shape[1], 9, 4).permute(0, 2, 1, 3).contiguous()  # [K][xi // 4][N][xi % 4]
        uw = torch.empty(36 * cin * cout, device=DEV)
        Wd = W.to(DEV)
        H.call("smc_wino4_weights_f32", Wd.data_ptr(), cout, cin, flip, uw.data_ptr(), H.stream())
        torch.cuda.synchronize()
        got = uw.cpu().double().reshape(ref.shape)
        assert (got - ref).abs().max().item() <= 2 ** -23 * ref.abs().max().item(), flip


@pytest.mark.parametrize("act,clamp", [("lrelu", 1.5), ("linear", -1.0)])
def test_wino4_modact_epilogue_vs_f2x2(act, clamp):
    """The MODACT forward of a SynthesisLayer conv1 (demod d, per-image noise, bias, activation, gain, clamp, u
    store) through F(4x4) and F(2x2): same epilogue function on u's within the conv tolerance."""
    from stylemc_amd import _hip as H, modconv
    n, c, r = 2, 64, 64
    g = torch.Generator().manual_seed(11)
    W = (torch.randn(c, c, 3, 3, generator=g) / (3 * c ** 0.5)).to(DEV)
    x = torch.randn(n, c, r, r, generator=g).to(DEV)
    s = (torch.rand(n, c, generator=g) + 0.5).to(DEV)
    d = (torch.rand(n, c, generator=g) + 0.5).to(DEV)
    noise = torch.randn(n, 1, r, r, generator=g).to(DEV)
    strength = torch.tensor([0.3], device=DEV)
    bias = torch.randn(c, generator=g).to(DEV)
    P = modconv.PackedConv(W, 1)
    outs = {}
    for name in ("wino4", "wino"):
        y = torch.empty(n, c, r, r, device=DEV)
        u = torch.empty_like(y)
        epi = modconv._epilogue(H.EPI_MODACT, d, noise, r * r, strength, bias, act, 0.2, 2 ** 0.5, clamp, u)
        if name == "wino4":
            modconv.wino4(x, y, P.wino4_weights(0), c, c, s=s, epi=epi)
        else:
            modconv.wino(x, y, P.wino_weights(0), c, c, s=s, epi=epi)
        outs[name] = (y, u)
    torch.cuda.synchronize()
    (y4, u4), (y2, u2) = outs["wino4"], outs["wino"]
    scale = u2.abs().max().item()
    assert (u4 - u2).abs().max().item() <= 5e-5 * scale
    assert (y4 - y2).abs().max().item() <= 2e-4 * y2.abs().max().item()
    assert ((y4 - y2).norm() / y2.norm()).item() <= 1e-5


def test_wino4_unsupported_shapes():
    H = _lib()
    lib = H.load()
    assert lib.smc_conv3x3_wino4_supported(1, 512, 512, 32, 32) == 0   # w < 64
    assert lib.smc_conv3x3_wino4_supported(1, 10, 64, 64, 64) == 0     # cin % 4
    assert lib.smc_conv3x3_wino4_supported(1, 32, 32, 64, 64) == 0     # cout % 64
    assert lib.smc_conv3x3_wino4_supported(1, 32, 64, 12, 64) == 0     # h % 8
    x = torch.zeros(1, 32, 32, 32, device=DEV)
    y = torch.zeros(1, 32, 32, 32, device=DEV)
    uw = torch.zeros(36 * 32 * 32, device=DEV)
    rc = lib.smc_conv3x3_wino4_f32(x.data_ptr(), 1, 32, 32, 32, y.data_ptr(), 32, uw.data_ptr(), None, None,
                                   H.stream())
    assert rc == 2 and b"F(4x4)" in lib.smc_last_error()
