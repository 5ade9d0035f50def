"""Small-plane Winograd F(2x2, 3x3) with split-K (csrc/wino_sp.hip) -- the IR-SE50 14x14 / 7x7 stage convs.

Against fp64 conv2d of the same fp32 inputs: every output within 2e-6 x sum |w x| (the F(2x2) bound of
tests/test_gpu_wino.py) for the raw conv (STORE), and the PRELU / AFFINE epilogues applied by the split-K reduction
against the same epilogue in fp64.  Taps come from a packed 9-tap phase (smc_wino_taps_f32), the form the IR-SE50
executor holds.
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


def _run(n, cin, cout, h, w, mode="store", seed=0):
    from stylemc_amd import _hip, modconv
    from stylemc_amd.irse_hip import fwd_taps
    g = torch.Generator().manual_seed(seed + n + cin + h)
    x = torch.randn(n, cin, h, w, generator=g)
    W = torch.randn(cout, cin, 3, 3, generator=g) / (3 * cin ** 0.5)
    taps, wk = fwd_taps(W.double())
    wkd = wk.to(DEV, torch.float32).contiguous()
    ph = modconv._phase(taps, 1, h, w, 0, 0, 1, 1, wkd)
    lib = _hip.load()
    assert lib.smc_wino_sp_supported(n, cin, cout, h, w) == 1
    uw = torch.empty(16 * cin * cout, device=DEV)
    _hip.call("smc_wino_taps_f32", ctypes.byref(ph), cin, cout, uw.data_ptr(), _hip.stream())
    ws_bytes = lib.smc_wino_sp_workspace_size(n, cin, cout, h, w)
    ws = torch.empty(ws_bytes // 4, device=DEV)
    y = torch.full((n, cout, h, w), float("nan"), device=DEV)
    sc = (torch.rand(cout, generator=g) + 0.5)
    bias = torch.randn(cout, generator=g)
    alpha = torch.rand(cout, generator=g) * 0.5
    u = torch.full_like(y, float("nan"))
    e = _hip.ConvEpilogue()
    e.act, e.gain, e.clamp = _hip.ACT_CODES["linear"], 1.0, -1.0
    keep = [sc.to(DEV), bias.to(DEV), alpha.to(DEV)]
    if mode == "store":
        e.mode = _hip.EPI_STORE
    elif mode == "prelu":
        e.mode, e.scale_c, e.bias, e.alpha_c, e.u_save = (_hip.EPI_PRELU, keep[0].data_ptr(), keep[1].data_ptr(),
                                                          keep[2].data_ptr(), u.data_ptr())
    else:
        e.mode, e.scale_c, e.bias = _hip.EPI_AFFINE, keep[0].data_ptr(), keep[1].data_ptr()
    xd = x.to(DEV)
    _hip.call("smc_conv3x3_wino_sp_f32", xd.data_ptr(), n, cin, h, w, y.data_ptr(), cout, uw.data_ptr(),
              ctypes.byref(e), ws.data_ptr(), ws_bytes, _hip.stream())
    torch.cuda.synchronize()
    ref = F.conv2d(x.double(), W.double(), padding=1)
    bound = F.conv2d(x.double().abs(), W.double().abs(), padding=1)
    return y.cpu().double(), u.cpu().double(), ref, bound, sc.double(), bias.double(), alpha.double()


SHAPES = [(4, 256, 256, 14, 14), (4, 512, 512, 7, 7), (3, 512, 512, 7, 7), (2, 64, 96, 16, 16), (5, 32, 64, 5, 6),
          (1, 16, 32, 2, 2)]


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_wino_sp_store_vs_fp64(shape):
    y, _, ref, bound, *_ = _run(*shape)
    assert torch.isfinite(y).all()
    ratio = ((y - ref).abs() / (bound + 1e-30)).max().item()
    assert ratio <= TOL, f"{shape}: max err / sum|w x| {ratio:.3e}"


@pytest.mark.parametrize("mode", ["prelu", "affine"])
def test_wino_sp_epilogue_modes(mode):
    y, u, ref, bound, sc, bias, alpha = _run(4, 256, 256, 14, 14, mode=mode, seed=5)
    z = ref * sc[None, :, None, None] + bias[None, :, None, None]
    zb = bound * sc[None, :, None, None]
    if mode == "prelu":
        assert ((u - z).abs() / (zb + 1e-30)).max().item() <= TOL
        expect = torch.where(z >= 0, z, z * alpha[None, :, None, None])
        # PReLU of a value within the conv tolerance of 0 may take the other branch: compare away from the kink
        away = (z.abs() > 4 * TOL * zb)
        assert ((y - expect).abs() / (zb + 1e-30))[away].max().item() <= TOL
    else:
        assert ((y - z).abs() / (zb + 1e-30)).max().item() <= TOL


def test_wino_sp_unsupported():
    from stylemc_amd import _hip
    lib = _hip.load()
    assert lib.smc_wino_sp_supported(4, 256, 256, 28, 28) == 0   # planes > 16x16
    assert lib.smc_wino_sp_supported(4, 12, 256, 14, 14) == 0    # cin % 8
    assert lib.smc_wino_sp_supported(4, 256, 48, 14, 14) == 0    # cout % 32
