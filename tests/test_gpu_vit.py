"""Parity of the HIP CLIP ViT kernels (through the C ABI) against fp64 / fp32 PyTorch references and the
CPU oracle's openai/CLIP VisionTransformer restatement (oracle/losses.py).

Tolerances (fp32 MFMA / VALU, different summation order):
  GEMM + epilogues: 2e-5 of max|ref| (fp64 reference); LayerNorm fwd/bwd: 2e-5; attention fwd 2e-5,
  bwd 5e-5; patch permutation: exact; whole ViT-B/32 forward: 1e-4 of max|ref| vs the oracle (CPU fp32),
  input gradient: 1e-3 of max|grad| and cosine >= 0.99999.
"""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def close(a, b, tol, what=""):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    scale = max(b.abs().max().item(), 1e-12)
    err = (a - b).abs().max().item()
    assert err <= tol * scale, f"{what}: max err {err:.3e} > {tol:.1e} * {scale:.3e}"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from stylemc_amd import build
    build.build(verbose=False)
    torch.backends.cuda.matmul.allow_tf32 = False


def _lin(a, w_km, epi=None, c=None):
    from stylemc_amd import _hip
    M, K = a.shape
    N = w_km.shape[1]
    c = torch.empty(M, N, device=DEV) if c is None else c
    wsb = _hip.load().smc_linear_workspace_size(M, N, K)
    ws = torch.empty(max(wsb // 4, 1), device=DEV)
    _hip.call("smc_linear_f32", a.data_ptr(), a.stride(0), w_km.data_ptr(), w_km.stride(0), c.data_ptr(), c.stride(0),
              M, N, K, ctypes.byref(epi) if epi is not None else None, ws.data_ptr(), wsb, _hip.stream())
    return c


def qgelu(x):
    return x * torch.sigmoid(1.702 * x)


def qgelu_grad(x):
    s = torch.sigmoid(1.702 * x)
    return s + 1.702 * x * s * (1 - s)


@pytest.mark.parametrize("M,N,K", [(200, 2304, 768), (200, 768, 3072), (200, 3072, 768), (196, 768, 3072),
                                   (4, 512, 768), (37, 132, 64), (1, 4, 32), (400, 768, 768)])
def test_linear_plain(M, N, K):
    g = torch.Generator().manual_seed(M * 7 + N + K)
    a = torch.randn(M, K, generator=g)
    w = torch.randn(K, N, generator=g) / K ** 0.5
    ref = a.double() @ w.double()
    close(_lin(a.to(DEV), w.to(DEV)), ref, 2e-5, f"linear {M}x{N}x{K}")


@pytest.mark.parametrize("M,N,K", [(200, 3072, 768), (200, 768, 3072), (50, 256, 96)])
def test_linear_epilogues(M, N, K):
    from stylemc_amd import _hip
    g = torch.Generator().manual_seed(11)
    a = torch.randn(M, K, generator=g)
    w = torch.randn(K, N, generator=g) / K ** 0.5
    bias = torch.randn(N, generator=g)
    res = torch.randn(M, N, generator=g)
    pre_in = torch.randn(M, N, generator=g)
    acc = a.double() @ w.double()
    ad, wd = a.to(DEV), w.to(DEV)
    # bias + QuickGELU, pre-activation saved
    pre = torch.empty(M, N, device=DEV)
    e = _hip.LinearEpilogue()
    bd = bias.to(DEV)
    e.bias, e.act, e.pre_save, e.ld_pre = bd.data_ptr(), _hip.LIN_ACT_QUICKGELU, pre.data_ptr(), N
    y = _lin(ad, wd, e)
    z = acc + bias.double()
    close(pre, z, 2e-5, "pre-activation")
    close(y, qgelu(z), 2e-5, "bias+quickgelu")
    # residual (in place: C aliases the residual) + bias
    c = res.clone().to(DEV)
    e = _hip.LinearEpilogue()
    e.bias, e.residual, e.ld_res = bd.data_ptr(), c.data_ptr(), N
    _lin(ad, wd, e, c=c)
    close(c, acc + bias.double() + res.double(), 2e-5, "bias+residual in place")
    # QuickGELU backward multiply
    pd = pre_in.to(DEV)
    e = _hip.LinearEpilogue()
    e.dact_pre, e.ld_dact = pd.data_ptr(), N
    close(_lin(ad, wd, e), acc * qgelu_grad(pre_in.double()), 2e-5, "dgelu")


def test_linear_rejects_bad_shapes():
    from stylemc_amd import _hip
    lib = _hip.load()
    a = torch.zeros(4, 48, device=DEV)
    rc = lib.smc_linear_f32(a.data_ptr(), 48, a.data_ptr(), 48, a.data_ptr(), 48, 4, 48, 48, None, None, 0, None)
    assert rc == 2 and b"K % 32" in lib.smc_last_error()


@pytest.mark.parametrize("rows,dim", [(200, 768), (7, 64), (4, 1024)])
def test_layernorm(rows, dim):
    from stylemc_amd import _hip
    g = torch.Generator().manual_seed(rows + dim)
    x = (torch.randn(rows, dim, generator=g) * 3 + 1).double()
    w = torch.randn(dim, generator=g).double()
    b = torch.randn(dim, generator=g).double()
    dy = torch.randn(rows, dim, generator=g).double()
    dres = torch.randn(rows, dim, generator=g).double()
    xr = x.clone().requires_grad_(True)
    y_ref = torch.nn.functional.layer_norm(xr, (dim,), w, b, 1e-5)
    (dx_ref,) = torch.autograd.grad(y_ref, xr, dy)
    xf, wf, bf = x.float().to(DEV), w.float().to(DEV), b.float().to(DEV)
    y = torch.empty(rows, dim, device=DEV)
    mean = torch.empty(rows, device=DEV)
    rstd = torch.empty(rows, device=DEV)
    _hip.call("smc_layernorm_fwd_f32", xf.data_ptr(), dim, wf.data_ptr(), bf.data_ptr(), y.data_ptr(), dim,
              mean.data_ptr(), rstd.data_ptr(), rows, dim, 1e-5, _hip.stream())
    close(y, y_ref, 2e-5, "ln fwd")
    close(mean, x.mean(1), 2e-5, "ln mean")
    dx = dres.float().to(DEV)  # in place: dx aliases the residual gradient
    dyf = dy.float().to(DEV)
    _hip.call("smc_layernorm_bwd_f32", dyf.data_ptr(), dim, xf.data_ptr(), dim, mean.data_ptr(), rstd.data_ptr(),
              wf.data_ptr(), dx.data_ptr(), dim, dx.data_ptr(), dim, rows, dim, _hip.stream())
    close(dx, dx_ref + dres, 2e-5, "ln bwd + residual")


def _attn_ref(qkv, B, L, H):
    D = H * 64
    q, k, v = qkv.view(B, L, 3, H, 64).permute(2, 0, 3, 1, 4).unbind(0)
    p = torch.softmax((q @ k.transpose(-1, -2)) * 0.125, dim=-1)
    o = (p @ v).transpose(1, 2).reshape(B * L, D)
    return o, p


@pytest.mark.parametrize("B,L,H", [(4, 50, 12), (2, 197, 12), (3, 7, 2), (1, 64, 1), (1, 65, 3)])
def test_attention(B, L, H):
    from stylemc_amd import _hip
    g = torch.Generator().manual_seed(B * L + H)
    D = H * 64
    qkv = torch.randn(B * L, 3 * D, generator=g, dtype=torch.float64)
    do = torch.randn(B * L, D, generator=g, dtype=torch.float64)
    qr = qkv.clone().requires_grad_(True)
    o_ref, p_ref = _attn_ref(qr, B, L, H)
    (dqkv_ref,) = torch.autograd.grad(o_ref, qr, do)
    qf = qkv.float().to(DEV)
    o = torch.empty(B * L, D, device=DEV)
    p = torch.empty(B, H, L, L, device=DEV)
    _hip.call("smc_attention_fwd_f32", qf.data_ptr(), o.data_ptr(), p.data_ptr(), B, L, H, 64, 0.125, _hip.stream())
    close(o, o_ref, 2e-5, "attn out")
    close(p, p_ref, 2e-5, "attn probs")
    dqkv = torch.full((B * L, 3 * D), float("nan"), device=DEV)
    dof = do.float().to(DEV)
    _hip.call("smc_attention_bwd_f32", dof.data_ptr(), qf.data_ptr(), p.data_ptr(), dqkv.data_ptr(), B, L, H, 64,
              0.125, _hip.stream())
    close(dqkv, dqkv_ref, 5e-5, "attn dqkv")


def test_attention_backward_deterministic():
    """L <= 64 uses two query blocks per head; their two adds onto zero commute -> bitwise repeatable."""
    from stylemc_amd import _hip
    B, L, H = 4, 50, 12
    g = torch.Generator().manual_seed(3)
    qkv = torch.randn(B * L, 3 * H * 64, generator=g).to(DEV)
    do = torch.randn(B * L, H * 64, generator=g).to(DEV)
    o = torch.empty(B * L, H * 64, device=DEV)
    p = torch.empty(B, H, L, L, device=DEV)
    _hip.call("smc_attention_fwd_f32", qkv.data_ptr(), o.data_ptr(), p.data_ptr(), B, L, H, 64, 0.125, _hip.stream())
    outs = []
    for _ in range(3):
        d = torch.empty(B * L, 3 * H * 64, device=DEV)
        _hip.call("smc_attention_bwd_f32", do.data_ptr(), qkv.data_ptr(), p.data_ptr(), d.data_ptr(), B, L, H, 64,
                  0.125, _hip.stream())
        outs.append(d)
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


def test_patch_permutation_roundtrip():
    from stylemc_amd import _hip
    img = torch.randn(2, 3, 224, 224, device=DEV)
    patches = torch.empty(2 * 49, 3 * 32 * 32, device=DEV)
    _hip.call("smc_patch_im2col_f32", img.data_ptr(), patches.data_ptr(), 2, 3, 7, 32, 0, _hip.stream())
    ref = img.reshape(2, 3, 7, 32, 7, 32).permute(0, 2, 4, 1, 3, 5).reshape(2 * 49, 3 * 32 * 32)
    assert torch.equal(patches, ref)
    back = torch.empty_like(img)
    _hip.call("smc_patch_im2col_f32", back.data_ptr(), patches.data_ptr(), 2, 3, 7, 32, 1, _hip.stream())
    assert torch.equal(back, img)


def _vit_pair(name, B, seed=4):
    from oracle import losses as OL
    from stylemc_amd import synthetic, vit_hip
    from stylemc_amd.clip_model import VIT_CONFIGS
    cfg = VIT_CONFIGS[name]
    hip = vit_hip.build_visual(name, seed=seed, device=DEV)
    ora = OL.CLIPVisual(**cfg).eval()
    ora.load_state_dict(synthetic.seeded_state_dict(ora, seed=seed))
    ora.requires_grad_(False)
    g = torch.Generator().manual_seed(B)
    x = torch.randn(B, 3, 224, 224, generator=g)
    cot = torch.randn(B, cfg["output_dim"], generator=g)
    return hip, ora, x, cot


@pytest.fixture(params=[True, False], ids=["x3", "fp32"])
def vit_x3(request, monkeypatch):
    """Both product forms of the tower's projections: split-bf16 (vit_hip.X3, the default) and exact-fp32 MFMA."""
    from stylemc_amd import vit_hip
    monkeypatch.setattr(vit_hip, "X3", request.param)
    return request.param


@pytest.mark.parametrize("name,B", [("ViT-B/32", 4), ("ViT-B/32", 1), ("ViT-B/32", 8), ("ViT-B/16", 2)])
def test_vit_forward_backward_vs_oracle(name, B, vit_x3):
    hip, ora, x, cot = _vit_pair(name, B)
    assert hip.cfg.products == (1 if vit_x3 else 0)
    xo = x.clone().requires_grad_(True)
    yo = ora(xo)
    (dxo,) = torch.autograd.grad(yo, xo, cot)
    xg = x.to(DEV).requires_grad_(True)
    yg = hip(xg)
    (dxg,) = torch.autograd.grad(yg, xg, cot.to(DEV))
    close(yg, yo, 1e-4, f"{name} B={B} embedding")
    close(dxg, dxo, 1e-3, f"{name} B={B} image gradient")
    cos = torch.nn.functional.cosine_similarity(dxg.cpu().double().flatten(), dxo.double().flatten(), dim=0)
    assert cos >= 0.99999, cos


def test_vit_no_grad_matches_grad_path_and_torch_impl():
    """no_grad forward (no saved activations) == grad-path forward bitwise; vs the PyTorch-ROCm tower 1e-4."""
    from stylemc_amd import clip_model
    hip, _, x, _ = _vit_pair("ViT-B/32", 4)
    xg = x.to(DEV)
    with torch.no_grad():
        y0 = hip(xg)
    y1 = hip(xg.clone().requires_grad_(True))
    assert torch.equal(y0, y1.detach())
    tv = clip_model.build_visual("ViT-B/32", seed=4, device=DEV)
    with torch.no_grad():
        close(y0, tv(xg), 1e-4, "hip vs torch tower")


@pytest.mark.parametrize("B,n", [(8, 4), (2, 1), (5, 3)])
def test_vit_partial_backward(B, n):
    """n_grad < B (batched [edited; original] pair): the gradient of the leading n images equals the
    full backward with a zero cotangent for the rest, and the rest get exactly zero."""
    hip, _, x, cot = _vit_pair("ViT-B/32", B)
    cot[n:] = 0
    xg = x.to(DEV).requires_grad_(True)
    (dfull,) = torch.autograd.grad(hip(xg), xg, cot.to(DEV))
    xp = x.to(DEV).requires_grad_(True)
    yp = hip(xp, n_grad=n)
    (dpart,) = torch.autograd.grad(yp, xp, cot.to(DEV))
    assert torch.count_nonzero(dpart[n:]) == 0
    close(dpart[:n], dfull[:n], 1e-4, f"B={B} n_grad={n} image gradient")


def test_clip_pair_loss_equals_separate_encodes():
    """CLIPLoss.per_sample_pair (one tower batch) == per_sample (two encodes), values and gradient."""
    from stylemc_amd import vit_hip
    from stylemc_amd.clip_loss import CLIPLoss
    hip = vit_hip.build_visual("ViT-B/32", seed=4, device=DEV)
    g = torch.Generator().manual_seed(1)
    text = torch.nn.functional.normalize(torch.randn(1, 512, generator=g), dim=1).to(DEV)
    cl = CLIPLoss(device=DEV, visual=hip, text_features=text)
    src = torch.randn(3, 3, 224, 224, generator=g).to(DEV)
    tgt = (src + 0.1 * torch.randn(src.shape, generator=g).to(DEV))
    t1 = tgt.clone().requires_grad_(True)
    l1 = cl.per_sample(src, t1)
    (g1,) = torch.autograd.grad(l1.sum(), t1)
    t2 = tgt.clone().requires_grad_(True)
    l2 = cl.per_sample_pair(t2, src)
    (g2,) = torch.autograd.grad(l2.sum(), t2)
    close(l2, l1, 1e-5, "pair vs separate loss")
    close(g2, g1, 1e-4, "pair vs separate gradient")


@pytest.mark.parametrize("res", [1024, 512, 256, 224])
def test_unprocess_kernel_vs_torch_ops(res):
    """UnprocessFn (smc_clip_unprocess_f32/_bwd_f32) == (img*127.5+128).clamp(0,255) -> F.interpolate bicubic
    (align_corners=False) -> (x/255 - mean)/std (find_direction.py:49-52) on the same GPU tensors; inputs
    scaled so that the clamp is active on part of the image."""
    import torch.nn.functional as F
    from stylemc_amd import utils
    from stylemc_amd.find_direction import UnprocessFn
    mean, std = utils.get_mean_std(DEV)
    g = torch.Generator().manual_seed(res)
    img = (1.3 * torch.randn(2, 3, res, res, generator=g)).to(DEV)
    cot = torch.randn(2, 3, 224, 224, generator=g).to(DEV)
    a = img.clone().requires_grad_(True)
    ya = UnprocessFn.apply(a, mean, std, 224)
    (da,) = torch.autograd.grad(ya, a, cot)
    b = img.clone().requires_grad_(True)
    x = (b * 127.5 + 128).clamp(0, 255)
    x = F.interpolate(x, size=(224, 224), mode="bicubic", align_corners=False)
    yb = (x / 255 - mean) / std
    (db,) = torch.autograd.grad(yb, b, cot)
    close(ya, yb, 1e-5, "unprocess")
    close(da, db, 1e-5, "unprocess gradient")
