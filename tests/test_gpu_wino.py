"""Winograd F(2x2, 3x3) conv kernel (csrc/wino.hip) through the C ABI.

Checked against fp64 conv2d on the same fp32 inputs.  Tolerance: the error of every output element is bounded by
2e-6 x sum_k |w_k x_k| (the fp64 conv of |W| and |x*s|): the direct fp32 implicit GEMM sits near 2^-24 x that sum
per product chain; the Winograd transforms (input / output adds, the 1/2 factors of G) add a few more roundings.
The MODACT epilogue (demod, noise, bias, lrelu, clamp, u store) is compared with the direct smc_conv_gemm_f32 path
on the same inputs (same epilogue function; outputs away from the lrelu / clamp kinks agree to the conv tolerance).
"""
import ctypes

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"
TOL = 2e-6


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
    assert ratio <= TOL, f"{what}: max err / sum|w x| = {ratio:.3e} > {TOL:.1e}"
    rel = ((got.double().cpu() - ref).norm() / ref.norm()).item()
    assert rel <= 1e-6, f"{what}: relative norm error {rel:.3e}"


SHAPES = [  # n, cin, cout, h, w  (TC 16 / 32 / 64 block shapes, non-square, 512 channels, cin != cout)
    (2, 32, 32, 32, 32),
    (1, 64, 64, 64, 64),
    (2, 16, 32, 128, 128),
    (1, 32, 64, 256, 128),
    (2, 512, 512, 32, 32),
    (1, 128, 96, 64, 256),
    (4, 32, 32, 1024, 1024),
]


@pytest.mark.parametrize("ws", [False, True], ids=["in_kernel_scale", "workspace"])
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_wino_forward_vs_fp64(shape, ws):
    """Style-scaled forward.  Without a workspace the kernel scales each transformed patch by s[n, c]; with the
    workspace smc_conv3x3_wino_workspace_size asks for, the 32..128-channel shapes take per-image U with s folded in
    (wino_ufold_kernel) and the 512-channel 32 x 32 one splits K."""
    H = _lib()
    n, cin, cout, h, w = shape
    g = torch.Generator().manual_seed(sum(shape))
    x = torch.randn(n, cin, h, w, generator=g)
    s = torch.rand(n, cin, generator=g) + 0.5
    W = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    assert H.load().smc_conv3x3_wino_supported(n, cin, cout, h, w) == 1
    xd, sd, Wd = x.to(DEV), s.to(DEV), W.to(DEV)
    uw = torch.empty(16 * cin * cout, device=DEV)
    H.call("smc_wino_weights_f32", Wd.data_ptr(), cout, cin, 0, uw.data_ptr(), H.stream())
    y = torch.empty(n, cout, h, w, device=DEV)
    if ws:
        nb = H.load().smc_conv3x3_wino_workspace_size(n, cin, cout, h, w)
        wsb = torch.full((max(nb // 4, 1),), float("nan"), device=DEV)
        H.call("smc_conv3x3_wino_ws_f32", xd.data_ptr(), n, cin, h, w, y.data_ptr(), cout, uw.data_ptr(),
               sd.data_ptr(), None, wsb.data_ptr(), nb, H.stream())
    else:
        H.call("smc_conv3x3_wino_f32", xd.data_ptr(), n, cin, h, w, y.data_ptr(), cout, uw.data_ptr(), sd.data_ptr(),
               None, H.stream())
    torch.cuda.synchronize()
    if n * h * w > 1 << 20:  # the 1024-px case: check two images' worth of rows (fp64 conv on CPU is slow)
        y, x, s = y[:, :, :64], x[:, :, :66], s
        ref_x = (x.double() * s.double()[:, :, None, None])
        got = y.cpu()
        ref = F.conv2d(ref_x, W.double(), padding=1)[:, :, :64]
        bound = F.conv2d(ref_x.abs(), W.double().abs(), padding=1)[:, :, :64]
        ratio = ((got.double() - ref).abs() / (bound + 1e-30)).max().item()
        assert ratio <= TOL, ratio
        return
    _check(y, x.double() * s.double()[:, :, None, None], W.double(), f"fwd {shape}")


@pytest.mark.parametrize("shape", SHAPES[:6], ids=lambda s: "x".join(map(str, s)))
def test_wino_data_grad_vs_fp64(shape):
    """flip = 1 weights: the conv^T of the 3x3 'same' conv (its data gradient) with cin / cout swapped."""
    H = _lib()
    n, cin, cout, h, w = shape
    g = torch.Generator().manual_seed(7 + sum(shape))
    gy = torch.randn(n, cout, h, w, generator=g)
    W = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    if not H.load().smc_conv3x3_wino_supported(n, cout, cin, h, w):
        pytest.skip("transposed shape has no Winograd kernel (cout % 32)")
    Wd = W.to(DEV)
    uw = torch.empty(16 * cin * cout, device=DEV)
    H.call("smc_wino_weights_f32", Wd.data_ptr(), cout, cin, 1, uw.data_ptr(), H.stream())
    dx = torch.empty(n, cin, h, w, device=DEV)
    gyd = gy.to(DEV)
    H.call("smc_conv3x3_wino_f32", gyd.data_ptr(), n, cout, h, w, dx.data_ptr(), cin, uw.data_ptr(), None, None,
           H.stream())
    torch.cuda.synchronize()
    # conv^T of a 3x3 pad-1 conv = conv with the taps flipped and in/out swapped
    Wt = W.double().flip(2, 3).transpose(0, 1).contiguous()
    _check(dx, gy.double(), Wt, f"dgrad {shape}")


def test_wino_weights_vs_fp64():
    H = _lib()
    cout, cin = 64, 32
    W = torch.randn(cout, cin, 3, 3, generator=torch.Generator().manual_seed(3))
    G = torch.tensor([[1, 0, 0], [0.5, 0.5, 0.5], [0.5, -0.5, 0.5], [0, 0, 1]], dtype=torch.float64)
    for flip in (0, 1):
        g = W.double() if flip == 0 else W.double().flip(2, 3).transpose(0, 1)  # [N][K][3][3]
        U = torch.einsum("ai,nkij,bj->knab", G, g, G)  # [K][N][a][b]
        ref = U.permute(0, 2, 1, 3).contiguous()       # -> [K][a = xi // 4][N][b = xi % 4]
        uw = torch.empty(16 * cin * cout, device=DEV)
        Wd = W.to(DEV)
        H.call("smc_wino_weights_f32", Wd.data_ptr(), cout, cin, flip, uw.data_ptr(), H.stream())
        torch.cuda.synchronize()
        got = uw.cpu().double().reshape(ref.shape)
        assert (got - ref).abs().max().item() <= 1e-6 * ref.abs().max().item(), flip


def test_wino_modact_epilogue_vs_direct_gemm():
    """The forward a SynthesisLayer conv1 issues (MODACT: demod d, per-image noise, bias, lrelu, gain, clamp, u
    store) through the Winograd kernel and through the direct implicit GEMM: same epilogue, conv tolerance."""
    from stylemc_amd import modconv
    H = _lib()
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
    for name in ("wino", "direct"):
        y = torch.empty(n, c, r, r, device=DEV)
        u = torch.empty_like(y)
        epi = modconv._epilogue(H.EPI_MODACT, d, noise, r * r, strength, bias, "lrelu", 0.2, 2 ** 0.5, 1.5, u)
        if name == "wino":
            modconv.wino(x, y, P.wino_weights(0), c, c, s=s, epi=epi)
        else:
            phases, nph, _, _ = P.fwd_phases(r, r)
            modconv.gemm(x, y, phases, nph, c, c, s=s, epi=epi)
        outs[name] = (y, u)
    torch.cuda.synchronize()
    (yw, uw_), (yd, ud) = outs["wino"], outs["direct"]
    scale = ud.abs().max().item()
    assert (uw_ - ud).abs().max().item() <= 2e-5 * scale
    # y: identical epilogue on u's that differ by a few ulps; away from the kinks the difference stays at that level
    assert (yw - yd).abs().max().item() <= 1e-4 * yd.abs().max().item()
    assert ((yw - yd).norm() / yd.norm()).item() <= 1e-6


SPLIT_SHAPES = [  # grids under 512 work items: the split-K form (K splits of >= 8 steps)
    (2, 512, 512, 32, 32),   # 128 items, 4 splits
    (4, 512, 512, 32, 32),   # the FFHQ-1024 batch-4 32 x 32 conv: 256 items, 2 splits
    (1, 128, 96, 64, 256),   # 192 items, 2 splits (16 steps)
]


@pytest.mark.parametrize("shape", SPLIT_SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_wino_split_k_vs_fp64(shape):
    """smc_conv3x3_wino_ws_f32 with its workspace: K splits + the epilogue kernel's reduction, STORE vs fp64 and the
    MODACT epilogue (demod, noise, bias, lrelu, gain, clamp, u store) vs the single-pass kernel."""
    H = _lib()
    lib = H.load()
    n, cin, cout, h, w = shape
    ws_bytes = lib.smc_conv3x3_wino_workspace_size(n, cin, cout, h, w)
    assert ws_bytes > 0
    g = torch.Generator().manual_seed(5 + sum(shape))
    x = torch.randn(n, cin, h, w, generator=g)
    s = torch.rand(n, cin, generator=g) + 0.5
    W = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    xd, sd, Wd = x.to(DEV), s.to(DEV), W.to(DEV)
    uw = torch.empty(16 * cin * cout, device=DEV)
    H.call("smc_wino_weights_f32", Wd.data_ptr(), cout, cin, 0, uw.data_ptr(), H.stream())
    ws = torch.full((ws_bytes // 4,), float("nan"), device=DEV)
    y = torch.empty(n, cout, h, w, device=DEV)
    H.call("smc_conv3x3_wino_ws_f32", xd.data_ptr(), n, cin, h, w, y.data_ptr(), cout, uw.data_ptr(), sd.data_ptr(),
           None, ws.data_ptr(), ws_bytes, H.stream())
    torch.cuda.synchronize()
    _check(y, x.double() * s.double()[:, :, None, None], W.double(), f"split fwd {shape}")

    from stylemc_amd import modconv
    d = (torch.rand(n, cout, generator=g) + 0.5).to(DEV)
    noise = torch.randn(n, 1, h, w, generator=g).to(DEV)
    strength = torch.tensor([0.3], device=DEV)
    bias = torch.randn(cout, generator=g).to(DEV)
    outs = []
    for split in (True, False):
        yy, uu = torch.empty(n, cout, h, w, device=DEV), torch.empty(n, cout, h, w, device=DEV)
        epi = modconv._epilogue(H.EPI_MODACT, d, noise, h * w, strength, bias, "lrelu", 0.2, 2 ** 0.5, 1.5, uu)
        H.call("smc_conv3x3_wino_ws_f32", xd.data_ptr(), n, cin, h, w, yy.data_ptr(), cout, uw.data_ptr(),
               sd.data_ptr(), ctypes.byref(epi), ws.data_ptr() if split else None, ws_bytes if split else 0,
               H.stream())
        outs.append((yy, uu))
    torch.cuda.synchronize()
    (ys, us), (y1, u1) = outs
    assert (us - u1).abs().max().item() <= 2e-5 * u1.abs().max().item()
    assert (ys - y1).abs().max().item() <= 1e-4 * y1.abs().max().item()
    assert ((ys - y1).norm() / y1.norm()).item() <= 1e-6


def test_wino_split_plan():
    lib = _lib().load()
    assert lib.smc_conv3x3_wino_workspace_size(4, 512, 512, 32, 32) == 2 * 4 * 512 * 32 * 32 * 4
    assert lib.smc_conv3x3_wino_workspace_size(2, 512, 512, 32, 32) == 4 * 2 * 512 * 32 * 32 * 4
    assert lib.smc_conv3x3_wino_workspace_size(4, 512, 512, 64, 64) == 0     # 1024 items: one pass
    assert lib.smc_conv3x3_wino_workspace_size(2, 32, 32, 32, 32) == 2 * 32 * 16 * 32 * 4  # no split; folded U
    assert lib.smc_conv3x3_wino_workspace_size(1, 512, 512, 16, 16) == 0     # no kernel


def test_wino_unsupported_shapes():
    H = _lib()
    lib = H.load()
    assert lib.smc_conv3x3_wino_supported(1, 512, 512, 16, 16) == 0   # w < 32
    assert lib.smc_conv3x3_wino_supported(1, 12, 32, 64, 64) == 0     # cin % 8
    assert lib.smc_conv3x3_wino_supported(1, 32, 48, 64, 64) == 0     # cout % 32
    x = torch.zeros(1, 32, 16, 16, device=DEV)
    y = torch.zeros(1, 32, 16, 16, device=DEV)
    uw = torch.zeros(16 * 32 * 32, device=DEV)
    rc = lib.smc_conv3x3_wino_f32(x.data_ptr(), 1, 32, 16, 16, y.data_ptr(), 32, uw.data_ptr(), None, None,
                                  H.stream())
    assert rc == 2 and b"Winograd" in lib.smc_last_error()


# The split-bf16 F(2x2) kernel (wino.hip wino_x3_kernel) is off in the product; these tests switch it on
# (smc_set_wino_x3) around each check.
X3_SHAPES = [  # cin = cout = 32 with 2 x 32 tile blocks (w % 64 == 0, h % 4 == 0): the split-bf16 kernel
    (2, 32, 32, 64, 64),
    (1, 32, 32, 128, 256),
    (3, 32, 32, 68, 128),
    (4, 32, 32, 1024, 1024),
]


@pytest.fixture
def x3_mode():
    """The split-bf16 F(2x2) enabled for one test (smc_set_wino_x3; off in the product: slower in the full step,
    profiles/r06/wino_x3/README)."""
    lib = _lib().load()
    prev = lib.smc_set_wino_x3(2)
    yield
    lib.smc_set_wino_x3(prev)


def _x3_ws(n, h, w):
    nb = _lib().load().smc_conv3x3_wino_workspace_size(n, 32, 32, h, w)
    assert nb == n * 16 * 3 * 2 * 4 * 16 * 8 * 2, "not the split-bf16 plan (96 KB of U planes per image)"
    return nb, torch.full((nb // 4,), float("nan"), device=DEV)


def _rows_check(got, x64, w64, what, rows=None):
    if rows is not None:  # the 1024-px case: the first rows of every image (fp64 conv on CPU is slow)
        got, x64 = got[:, :, :rows], x64[:, :, :rows + 2]
    ref = F.conv2d(x64, w64, padding=1)
    bound = F.conv2d(x64.abs(), w64.abs(), padding=1)
    if rows is not None:
        ref, bound = ref[:, :, :rows], bound[:, :, :rows]
    ratio = ((got.double().cpu() - ref).abs() / (bound + 1e-30)).max().item()
    assert ratio <= TOL, f"{what}: max err / sum|w x| = {ratio:.3e} > {TOL:.1e}"


@pytest.mark.parametrize("shape", X3_SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_wino_x3_vs_fp64(shape, x3_mode):
    """The split-bf16 F(2x2) kernel (wino_x3_kernel, taken by the conv1 forward's MODACT form): the style-scaled
    forward (s folded into per-image planes) and a data-gradient-shaped call (flipped taps, one plane set), through that
    form with d = 1, no noise, no bias, lrelu slope 1, gain 1 and an unreachable clamp (y = the conv exactly), against
    fp64 at the fp32 kernel's tolerance TOL -- the three-term products leave out <= 2^-23 |u v| each."""
    from stylemc_amd import modconv
    H = _lib()
    plain = modconv._epilogue(H.EPI_MODACT, None, None, 0, None, None, "lrelu", 1.0, 1.0, 1e30, None)
    n, cin, cout, h, w = shape
    g = torch.Generator().manual_seed(13 + sum(shape))
    x = torch.randn(n, cin, h, w, generator=g)
    s = torch.rand(n, cin, generator=g) + 0.5
    W = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    nb, ws = _x3_ws(n, h, w)
    xd, sd, Wd = x.to(DEV), s.to(DEV), W.to(DEV)
    rows = 64 if h * w > 1 << 18 else None
    for flip in (0, 1):
        uw = torch.empty(16 * cin * cout, device=DEV)
        H.call("smc_wino_weights_f32", Wd.data_ptr(), cout, cin, flip, uw.data_ptr(), H.stream())
        y = torch.full((n, cout, h, w), float("nan"), device=DEV)
        H.call("smc_conv3x3_wino_ws_f32", xd.data_ptr(), n, cin, h, w, y.data_ptr(), cout, uw.data_ptr(),
               sd.data_ptr() if flip == 0 else None, ctypes.byref(plain), ws.data_ptr(), nb, H.stream())
        torch.cuda.synchronize()
        assert torch.isfinite(y).all()
        if flip == 0:
            _rows_check(y, x.double() * s.double()[:, :, None, None], W.double(), f"x3 fwd {shape}", rows)
        else:
            _rows_check(y, x.double(), W.double().flip(2, 3).transpose(0, 1).contiguous(), f"x3 dgrad {shape}", rows)


@pytest.mark.parametrize("act", ["lrelu", "linear"])
def test_wino_x3_modact_vs_fp32_kernel(act, x3_mode):
    """The MODACT epilogue through the split-bf16 kernel (workspace) and the fp32 F(2x2) kernel (no workspace): the
    conv1 forward form (lrelu, gain, clamp, noise, u store) and the data gradient's linear x d form."""
    from stylemc_amd import modconv
    H = _lib()
    n, c, h, w = 2, 32, 64, 128
    g = torch.Generator().manual_seed(17)
    W = (torch.randn(c, c, 3, 3, generator=g) / (3 * c ** 0.5)).to(DEV)
    x = torch.randn(n, c, h, w, generator=g).to(DEV)
    s = (torch.rand(n, c, generator=g) + 0.5).to(DEV)
    d = (torch.rand(n, c, generator=g) + 0.5).to(DEV)
    noise = torch.randn(n, 1, h, w, generator=g).to(DEV)
    strength = torch.tensor([0.3], device=DEV)
    bias = torch.randn(c, generator=g).to(DEV)
    P = modconv.PackedConv(W, 1)
    nb, ws = _x3_ws(n, h, w)
    outs = []
    for use_ws in (True, False):
        y, u = torch.empty(n, c, h, w, device=DEV), torch.empty(n, c, h, w, device=DEV)
        if act == "lrelu":
            epi = modconv._epilogue(H.EPI_MODACT, d, noise, h * w, strength, bias, "lrelu", 0.2, 2 ** 0.5, 1.5, u)
            sp = s.data_ptr()
        else:
            epi = modconv._epilogue(H.EPI_MODACT, d, None, 0, None, None, "linear", 0.0, 1.0, -1.0, u)
            sp = None
        H.call("smc_conv3x3_wino_ws_f32", x.data_ptr(), n, c, h, w, y.data_ptr(), c,
               P.wino_weights(0 if act == "lrelu" else 1).data_ptr(), sp, ctypes.byref(epi),
               ws.data_ptr() if use_ws else None, nb if use_ws else 0, H.stream())
        outs.append((y, u))
    torch.cuda.synchronize()
    (yx, ux), (yf, uf) = outs
    assert (ux - uf).abs().max().item() <= 2e-5 * uf.abs().max().item()
    assert (yx - yf).abs().max().item() <= 1e-4 * yf.abs().max().item()
    assert ((yx - yf).norm() / yf.norm()).item() <= 1e-6
