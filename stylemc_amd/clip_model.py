"""CLIP image tower (OpenAI ``VisionTransformer`` layout) for the directional CLIP loss.

The reference calls the third-party openai/CLIP package (clip_loss.py:11-13,21,25-26; not vendored,
unpinned git HEAD per male2female.ipynb).  This module keeps its state_dict layout (``conv1``,
``class_embedding``, ``positional_embedding``, ``ln_pre``, ``transformer.resblocks.{i}.{ln_1,attn,
ln_2,mlp.c_fc,mlp.c_proj}``, ``ln_post``, ``proj``) so real ``visual.*`` weights load unchanged, and
runs on PyTorch-ROCm in fp32 (BASELINE config 2: "CLIP on PyTorch-ROCm"): fused QKV projection +
``scaled_dot_product_attention`` per block.  ViT-B/32: patch 32, width 768, 12 layers, 12 heads,
output 512 (8.82 GFLOP per 224x224 image); ViT-B/16 for ``clip_type='large'``.
"""
import torch
import torch.nn.functional as F
from torch import nn

VIT_CONFIGS = {
    "ViT-B/32": dict(input_resolution=224, patch_size=32, width=768, layers=12, heads=12, output_dim=512),
    "ViT-B/16": dict(input_resolution=224, patch_size=16, width=768, layers=12, heads=12, output_dim=512),
}


class _Attention(nn.Module):
    """nn.MultiheadAttention-compatible parameters (in_proj_weight/bias, out_proj), batch-first compute."""

    def __init__(self, d, heads):
        super().__init__()
        self.heads = heads
        self.in_proj_weight = nn.Parameter(torch.empty(3 * d, d))
        self.in_proj_bias = nn.Parameter(torch.zeros(3 * d))
        self.out_proj = nn.Linear(d, d)

    def forward(self, x):  # x: [B, L, D]
        b, l, d = x.shape
        qkv = F.linear(x, self.in_proj_weight, self.in_proj_bias).view(b, l, 3, self.heads, d // self.heads)
        q, k, v = qkv.permute(2, 0, 3, 1, 4).unbind(0)
        o = F.scaled_dot_product_attention(q, k, v)
        return self.out_proj(o.transpose(1, 2).reshape(b, l, d))


class _Block(nn.Module):
    def __init__(self, d, heads):
        super().__init__()
        self.attn = _Attention(d, heads)
        self.ln_1 = nn.LayerNorm(d)
        self.mlp = nn.Sequential()
        self.mlp.add_module("c_fc", nn.Linear(d, 4 * d))
        self.mlp.add_module("gelu", _QuickGELU())
        self.mlp.add_module("c_proj", nn.Linear(4 * d, d))
        self.ln_2 = nn.LayerNorm(d)

    def forward(self, x):
        x = x + self.attn(self.ln_1(x))
        return x + self.mlp(self.ln_2(x))


class _QuickGELU(nn.Module):
    def forward(self, x):
        return x * torch.sigmoid(1.702 * x)


class _Transformer(nn.Module):
    def __init__(self, width, layers, heads):
        super().__init__()
        self.resblocks = nn.Sequential(*[_Block(width, heads) for _ in range(layers)])

    def forward(self, x):
        return self.resblocks(x)


class VisionTransformer(nn.Module):
    def __init__(self, input_resolution=224, patch_size=32, width=768, layers=12, heads=12, output_dim=512):
        super().__init__()
        self.input_resolution = input_resolution
        self.conv1 = nn.Conv2d(3, width, kernel_size=patch_size, stride=patch_size, bias=False)
        scale = width ** -0.5
        self.class_embedding = nn.Parameter(scale * torch.randn(width))
        self.positional_embedding = nn.Parameter(scale * torch.randn((input_resolution // patch_size) ** 2 + 1, width))
        self.ln_pre = nn.LayerNorm(width)
        self.transformer = _Transformer(width, layers, heads)
        self.ln_post = nn.LayerNorm(width)
        self.proj = nn.Parameter(scale * torch.randn(width, output_dim))

    def patch_embed(self, x):
        """conv1 with kernel == stride and no padding is a GEMM over non-overlapping patches:
        [B, grid^2, 3*p*p] @ W^T.  (MIOpen's backward-data for the 32x32/s32 conv spends ~200 s
        tuning on a fresh box per batch size; this form has no such cost.)"""
        b, c, h, w = x.shape
        p = self.conv1.kernel_size[0]
        g_h, g_w = h // p, w // p
        patches = x.reshape(b, c, g_h, p, g_w, p).permute(0, 2, 4, 1, 3, 5).reshape(b, g_h * g_w, c * p * p)
        return patches @ self.conv1.weight.reshape(self.conv1.out_channels, -1).t()

    def forward(self, x):
        x = self.patch_embed(x)                                           # [B, grid^2, width]
        cls = self.class_embedding.to(x.dtype).expand(x.shape[0], 1, -1)
        x = torch.cat([cls, x], dim=1) + self.positional_embedding.to(x.dtype)
        x = self.transformer(self.ln_pre(x))
        return self.ln_post(x[:, 0, :]) @ self.proj

    def flops_per_image(self):
        """Dense MACs x 2 of one forward (SURVEY.md section 8(d) accounting)."""
        w = self.conv1.out_channels
        p = self.conv1.kernel_size[0]
        g = (self.input_resolution // p) ** 2
        L = g + 1
        n_layers = len(self.transformer.resblocks)
        patch = 2 * g * 3 * p * p * w
        per_layer = 2 * L * w * 3 * w + 2 * 2 * L * L * w + 2 * L * w * w + 2 * 2 * L * w * 4 * w
        return patch + n_layers * per_layer + 2 * w * self.proj.shape[1]


def build_visual(name="ViT-B/32", state_dict=None, seed=0, device="cuda"):
    from . import synthetic
    model = VisionTransformer(**VIT_CONFIGS[name])
    model.load_state_dict(state_dict if state_dict is not None else synthetic.seeded_state_dict(model, seed=seed))
    return model.eval().requires_grad_(False).to(device)
