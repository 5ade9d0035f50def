"""CLIP ViT image tower on hand-written gfx950 kernels (BASELINE config 4: attention + MLP on MFMA HIP).

Drop-in for the third-party openai/CLIP ``VisionTransformer`` that the reference reaches through
``CLIPLoss.encode_image`` (clip_loss.py:21,25-26): same constructor arguments and state_dict keys as
:class:`stylemc_amd.clip_model.VisionTransformer` (``conv1``, ``class_embedding``,
``positional_embedding``, ``ln_pre``, ``transformer.resblocks.{i}.{ln_1, attn.in_proj_*,
attn.out_proj, ln_2, mlp.c_fc, mlp.c_proj}``, ``ln_post``, ``proj``), so ``visual.*`` weights load
unchanged.  The whole tower -- patch GEMM, 12 x (LN, QKV GEMM, attention, out-proj GEMM + residual,
LN, c_fc GEMM + QuickGELU, c_proj GEMM + residual), ln_post, projection -- runs as one native call
(``smc_vit_forward_f32``), and its data gradient as another (``smc_vit_backward_f32``); the C++ executor
inside the library launches the kernels on the caller's stream.  Weights are frozen (the reference's
loss only needs d loss / d image), so there are no weight gradients.

The frozen weights are packed once into one device buffer in the layout ``include/stylemc_hip.h``
documents (each projection stored K-major twice: W^T for the forward product, W for its adjoint).
"""
import torch
from torch import nn

from . import _hip
from .clip_model import VIT_CONFIGS, VisionTransformer

_ALIGN = 64


def _pad(t):
    t = t.detach().to(torch.float32).contiguous().reshape(-1)
    n = (t.numel() + _ALIGN - 1) // _ALIGN * _ALIGN
    if n == t.numel():
        return t
    return torch.cat([t, t.new_zeros(n - t.numel())])


# Split-bf16 products for the tower's projections (smc_vit_config.products = 1: three bf16 terms per fp32 operand, the
# six products above 2^-23 |a b|; the weights' planes are built once at packing).  Off by default: at 200..400 tokens
# the projections are bound by re-reading the weights, and the planes are 1.5x the fp32 bytes -- measured 451.6 vs
# 455.1 images/s with them on (profiles/r04/vit_ab/).  Module switch: tests run both forms.
X3 = False


def vit_config(width, layers, heads, patch, grid, out_dim, in_ch=3, ln_eps=1e-5, products=None):
    c = _hip.VitConfig()
    c.width, c.layers, c.heads, c.patch, c.grid, c.out_dim, c.in_ch, c.ln_eps = (width, layers, heads, patch, grid,
                                                                                  out_dim, in_ch, ln_eps)
    c.products = (1 if X3 else 0) if products is None else int(products)
    return c


def pack_weights(state_dict, layers):
    """The packed buffer of include/stylemc_hip.h (smc_vit_packed_floats order), as a flat fp32 tensor."""
    sd = {k: v.detach().to(torch.float32) for k, v in state_dict.items()}
    conv = sd["conv1.weight"]
    D = conv.shape[0]
    conv2 = conv.reshape(D, -1)
    segs = [conv2.t(), conv2, sd["class_embedding"], sd["positional_embedding"], sd["ln_pre.weight"],
            sd["ln_pre.bias"]]
    for i in range(layers):
        p = f"transformer.resblocks.{i}."
        w_in, w_out = sd[p + "attn.in_proj_weight"], sd[p + "attn.out_proj.weight"]
        w_fc, w_pr = sd[p + "mlp.c_fc.weight"], sd[p + "mlp.c_proj.weight"]
        segs += [sd[p + "ln_1.weight"], sd[p + "ln_1.bias"], w_in.t(), w_in, sd[p + "attn.in_proj_bias"],
                 w_out.t(), w_out, sd[p + "attn.out_proj.bias"], sd[p + "ln_2.weight"], sd[p + "ln_2.bias"],
                 w_fc.t(), w_fc, sd[p + "mlp.c_fc.bias"], w_pr.t(), w_pr, sd[p + "mlp.c_proj.bias"]]
    segs += [sd["ln_post.weight"], sd["ln_post.bias"], sd["proj"], sd["proj"].t()]
    return torch.cat([_pad(s) for s in segs])


class _VitFn(torch.autograd.Function):
    """Whole-tower forward / data gradient.  n_grad < batch: only the leading n_grad images are
    differentiated (the rest of the batch -- the original images of a batched pair -- get a zero gradient
    without being back-propagated)."""

    @staticmethod
    def forward(ctx, image, mod, n_grad):
        if not image.is_cuda:
            raise RuntimeError("HipVisionTransformer runs on the GPU only (got a CPU tensor)")
        image = image.to(torch.float32).contiguous()
        B = image.shape[0]
        exp = (mod.in_ch, mod.input_resolution, mod.input_resolution)
        if tuple(image.shape[1:]) != exp:
            raise ValueError(f"HipVisionTransformer expects [B, {exp[0]}, {exp[1]}, {exp[2]}], got {tuple(image.shape)}")
        lib = _hip.load()
        cfg = ctypes_ref(mod.cfg)
        out = torch.empty(B, mod.out_dim, device=image.device, dtype=torch.float32)
        saved = None
        if ctx.needs_input_grad[0]:
            saved = torch.empty(lib.smc_vit_saved_floats(cfg, B), device=image.device, dtype=torch.float32)
        ws_bytes = lib.smc_vit_workspace_bytes(cfg, B)
        ws = torch.empty(ws_bytes // 4, device=image.device, dtype=torch.float32)
        _hip.call("smc_vit_forward_f32", cfg, mod.packed.data_ptr(), image.data_ptr(), B, out.data_ptr(),
                  _hip.ptr(saved), ws.data_ptr(), ws_bytes, _hip.stream())
        ctx.mod, ctx.saved_buf, ctx.shape = mod, saved, image.shape
        ctx.n_grad = B if n_grad is None else int(n_grad)
        if not 1 <= ctx.n_grad <= B:
            raise ValueError(f"n_grad {n_grad} not in [1, {B}]")
        return out

    @staticmethod
    def backward(ctx, gout):
        mod, saved = ctx.mod, ctx.saved_buf
        B, nr = ctx.shape[0], ctx.n_grad
        gout = gout[:nr].to(torch.float32).contiguous()
        lib = _hip.load()
        cfg = ctypes_ref(mod.cfg)
        dimage = (torch.empty if nr == B else torch.zeros)(ctx.shape, device=gout.device, dtype=torch.float32)
        ws_bytes = lib.smc_vit_workspace_bytes(cfg, B)
        ws = torch.empty(ws_bytes // 4, device=gout.device, dtype=torch.float32)
        _hip.call("smc_vit_backward_f32", cfg, mod.packed.data_ptr(), gout.data_ptr(), B, nr, saved.data_ptr(),
                  dimage.data_ptr(), ws.data_ptr(), ws_bytes, _hip.stream())
        ctx.saved_buf = None
        return dimage, None, None


def vit_config_like(cfg, **kw):
    """A copy of a VitConfig with some fields replaced."""
    c = _hip.VitConfig()
    for name, _ in _hip.VitConfig._fields_:
        setattr(c, name, kw.get(name, getattr(cfg, name)))
    return c


def ctypes_ref(cfg):
    import ctypes
    return ctypes.byref(cfg)


class HipVisionTransformer(nn.Module):
    """openai/CLIP VisionTransformer (state_dict-compatible) executed by the gfx950 kernel library."""

    def __init__(self, input_resolution=224, patch_size=32, width=768, layers=12, heads=12, output_dim=512):
        super().__init__()
        # the parameters live in a regular VisionTransformer (state_dict keys, .to(), introspection);
        # the kernels read the packed copy, rebuilt by refresh() whenever weights are loaded
        self.tower = VisionTransformer(input_resolution, patch_size, width, layers, heads, output_dim)
        self.input_resolution = input_resolution
        self.in_ch = 3
        self.out_dim = output_dim
        self.layers = layers
        self.cfg = vit_config(width, layers, heads, patch_size, input_resolution // patch_size, output_dim)
        self.register_buffer("packed", torch.empty(0), persistent=False)

    # state_dict keys are the tower's own (visual.* layout), not prefixed by "tower."
    def state_dict(self, *args, **kwargs):
        return self.tower.state_dict(*args, **kwargs)

    def load_state_dict(self, state_dict, strict=True, assign=False):
        r = self.tower.load_state_dict(state_dict, strict=strict, assign=assign)
        self.refresh()
        return r

    def refresh(self):
        """Re-pack the frozen weights (after loading or moving them)."""
        packed = pack_weights(self.tower.state_dict(), self.layers)
        lib = _hip.load()
        dev = self.tower.proj.device
        if self.cfg.products == 1 and dev.type != "cuda":
            self.cfg.products = 0  # (planes are built on the GPU; a CPU-resident tower keeps the fp32 layout)
        fp32_part = lib.smc_vit_packed_floats(ctypes_ref(vit_config_like(self.cfg, products=0)))
        if fp32_part != packed.numel():
            raise RuntimeError(f"packed ViT weights: {packed.numel()} floats, the library expects {fp32_part}")
        n = lib.smc_vit_packed_floats(ctypes_ref(self.cfg))
        buf = torch.zeros(n, device=dev, dtype=torch.float32)
        buf[:fp32_part].copy_(packed)
        if self.cfg.products == 1:
            _hip.call("smc_vit_pack_x3", ctypes_ref(self.cfg), buf.data_ptr(), _hip.stream())
            torch.cuda.current_stream(dev).synchronize()
        self.packed = buf
        return self

    def flops_per_image(self):
        return self.tower.flops_per_image()

    supports_partial_grad = True

    def forward(self, image, n_grad=None):
        """n_grad: differentiate only the leading n_grad images of the batch (see _VitFn)."""
        if self.packed.numel() == 0:
            self.refresh()
        return _VitFn.apply(image, self, n_grad)


def build_visual(name="ViT-B/32", state_dict=None, seed=0, device="cuda"):
    from . import synthetic
    model = HipVisionTransformer(**VIT_CONFIGS[name])
    sd = state_dict if state_dict is not None else synthetic.seeded_state_dict(model.tower, seed=seed)
    model.tower.load_state_dict(sd)
    model = model.eval().requires_grad_(False).to(device)
    return model.refresh()
