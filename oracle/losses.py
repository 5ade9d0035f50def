"""CPU restatement of StyleMC's losses and loss composition (TEST ORACLE ONLY).

  unprocess / get_mean_std  <- find_direction.py:49-52, utils.py:90-97, torchvision 0.8 tensor
                               Resize(224, BICUBIC)+CenterCrop(224) (find_direction.py:258):
                               F.interpolate(bicubic, align_corners=False), no antialias
                               (torchvision is absent here -> parity unpinned for this step).
  CLIPVisual                <- third-party openai/CLIP ``model.VisionTransformer`` (not vendored,
                               called at clip_loss.py:21,25-26): ViT-B/32, QuickGELU, ln_pre,
                               CLS ln_post, projection.  PARITY UNPINNED vs the reference.
  CLIPLoss                  <- clip_loss.py:7-34 (directional loss)
  IRSE50 / IDLoss           <- id_loss/model_irse.py:10-49, id_loss/helpers.py:29-119,
                               id_loss/id_loss.py:7-39
  compute_loss              <- find_direction.py:172-200 (landmarks coefficient 0: that branch runs
                               under torch.no_grad, find_direction.py:90, and adds no gradient);
                               clip_loss_type 'nada' / 'nada_global' <- :100-114,150-157
  nada_preprocess / CLIPLossNADA <- clip_loss_nada.py:72-75 (torchvision Normalize(-1, 2) + CLIP Resize /
                               CenterCrop / Normalize, restated -> parity unpinned for that step),
                               :126-153 (template text direction), :177-229 (directional, angle, global
                               losses), :324-346 (forward)
"""
import math

import torch
import torch.nn.functional as F
from torch import nn

CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)


def get_mean_std(device="cpu"):
    mean = torch.tensor(CLIP_MEAN, dtype=torch.float32, device=device).view(-1, 1, 1)
    std = torch.tensor(CLIP_STD, dtype=torch.float32, device=device).view(-1, 1, 1)
    return mean, std


def resize_center_crop(x, size=224):
    h, w = x.shape[-2:]
    if h <= w:
        nh, nw = size, int(size * w / h)
    else:
        nh, nw = int(size * h / w), size
    x = F.interpolate(x, size=(nh, nw), mode="bicubic", align_corners=False)
    top = int(round((nh - size) / 2.0))
    left = int(round((nw - size) / 2.0))
    return x[..., top:top + size, left:left + size]


def unprocess(img, mean, std, size=224):
    x = (img * 127.5 + 128).clamp(0, 255)
    return (resize_center_crop(x, size) / 255 - mean) / std


# ----------------------------------------------------------------------------- CLIP ViT


class _LayerNorm(nn.LayerNorm):
    def forward(self, x):
        return super().forward(x.float()).to(x.dtype)


class _QuickGELU(nn.Module):
    def forward(self, x):
        return x * torch.sigmoid(1.702 * x)


class _ResBlock(nn.Module):
    def __init__(self, d, heads):
        super().__init__()
        self.attn = nn.MultiheadAttention(d, heads)
        self.ln_1 = _LayerNorm(d)
        self.mlp = nn.Sequential()
        self.mlp.add_module("c_fc", nn.Linear(d, 4 * d))
        self.mlp.add_module("gelu", _QuickGELU())
        self.mlp.add_module("c_proj", nn.Linear(4 * d, d))
        self.ln_2 = _LayerNorm(d)

    def forward(self, x):  # x: [L, N, D]
        h = self.ln_1(x)
        x = x + self.attn(h, h, h, need_weights=False)[0]
        return x + self.mlp(self.ln_2(x))


class _Transformer(nn.Module):
    def __init__(self, width, layers, heads):
        super().__init__()
        self.resblocks = nn.Sequential(*[_ResBlock(width, heads) for _ in range(layers)])

    def forward(self, x):
        return self.resblocks(x)


class CLIPVisual(nn.Module):
    """openai/CLIP VisionTransformer; ViT-B/32 by default (state_dict keys == ``visual.*``)."""

    def __init__(self, input_resolution=224, patch_size=32, width=768, layers=12, heads=12, output_dim=512):
        super().__init__()
        self.input_resolution = input_resolution
        self.conv1 = nn.Conv2d(3, width, kernel_size=patch_size, stride=patch_size, bias=False)
        scale = width ** -0.5
        self.class_embedding = nn.Parameter(scale * torch.randn(width))
        self.positional_embedding = nn.Parameter(scale * torch.randn((input_resolution // patch_size) ** 2 + 1, width))
        self.ln_pre = _LayerNorm(width)
        self.transformer = _Transformer(width, layers, heads)
        self.ln_post = _LayerNorm(width)
        self.proj = nn.Parameter(scale * torch.randn(width, output_dim))

    def forward(self, x):
        x = self.conv1(x)
        x = x.flatten(2).permute(0, 2, 1)
        cls = self.class_embedding.to(x.dtype).expand(x.shape[0], 1, -1)
        x = torch.cat([cls, x], dim=1) + self.positional_embedding.to(x.dtype)
        x = self.ln_pre(x).permute(1, 0, 2)
        x = self.transformer(x).permute(1, 0, 2)
        return self.ln_post(x[:, 0, :]) @ self.proj


class _TextResBlock(_ResBlock):
    def __init__(self, d, heads, mask):
        super().__init__(d, heads)
        self.register_buffer("attn_mask", mask, persistent=False)

    def forward(self, x):  # x: [L, N, D]
        h = self.ln_1(x)
        x = x + self.attn(h, h, h, need_weights=False, attn_mask=self.attn_mask)[0]
        return x + self.mlp(self.ln_2(x))


class CLIPText(nn.Module):
    """openai/CLIP text encoder (model.py encode_text; third-party, PARITY UNPINNED): token + positional
    embedding, residual blocks under the causal mask (build_attention_mask: -inf above the diagonal),
    ln_final, the EOT token's row (text.argmax(-1)) @ text_projection.  Keys == the CLIP model's text keys."""

    def __init__(self, embed_dim=512, context_length=77, vocab_size=49408, width=512, heads=8, layers=12):
        super().__init__()
        mask = torch.full((context_length, context_length), float("-inf")).triu_(1)
        self.token_embedding = nn.Embedding(vocab_size, width)
        self.positional_embedding = nn.Parameter(torch.empty(context_length, width))
        self.transformer = nn.Module()
        self.transformer.resblocks = nn.Sequential(*[_TextResBlock(width, heads, mask) for _ in range(layers)])
        self.ln_final = _LayerNorm(width)
        self.text_projection = nn.Parameter(torch.empty(width, embed_dim))

    def forward(self, text):
        x = self.token_embedding(text) + self.positional_embedding
        x = self.transformer.resblocks(x.permute(1, 0, 2)).permute(1, 0, 2)
        x = self.ln_final(x)
        return x[torch.arange(x.shape[0]), text.argmax(dim=-1)] @ self.text_projection


def text_features(text_model, tokens_pos, tokens_neg):
    """clip_loss.py:15-18: norm(E_T(pos) - E_T(neg))."""
    t = text_model(tokens_pos) - text_model(tokens_neg)
    return t / t.norm(dim=1, keepdim=True)


class CLIPLoss(nn.Module):
    """Directional CLIP loss (clip_loss.py:24-34) around an image encoder and a text direction."""

    def __init__(self, visual, text_direction):
        super().__init__()
        self.visual = visual
        t = text_direction.reshape(1, -1).float()
        self.register_buffer("text_features", t / t.norm(dim=1, keepdim=True))

    def forward(self, src_image, tgt_image):
        f = self.visual(tgt_image) - self.visual(src_image)
        f = f / f.norm(dim=1, keepdim=True)
        cos = F.cosine_similarity(f, self.text_features)
        return (len(src_image) - cos.sum()) / len(src_image)


# ----------------------------------------------------------------------------- StyleGAN-NADA losses


NADA_TEMPLATES = [
    'a photo of a {}.', 'a rendering of a {}.', 'a cropped photo of the {}.', 'the photo of a {}.',
    'a photo of a clean {}.', 'a photo of a dirty {}.', 'a dark photo of the {}.', 'a photo of my {}.',
    'a photo of the cool {}.', 'a close-up photo of a {}.', 'a bright photo of the {}.', 'a cropped photo of a {}.',
    'a photo of the {}.', 'a good photo of the {}.', 'a photo of one {}.', 'a close-up photo of the {}.',
    'a rendition of the {}.', 'a photo of the clean {}.', 'a rendition of a {}.', 'a photo of a nice {}.',
    'a good photo of a {}.', 'a photo of the nice {}.', 'a photo of the small {}.', 'a photo of the weird {}.',
    'a photo of the large {}.', 'a photo of a cool {}.', 'a photo of a small {}.',
]


def nada_preprocess(img, mean, std, size=224):
    """clip_loss_nada.py:72-75: Normalize(mean=-1, std=2) -> Resize(size, BICUBIC) -> CenterCrop -> Normalize."""
    x = (img - (-1.0)) / 2.0
    return (resize_center_crop(x, size) - mean) / std


class CLIPLossNADA(nn.Module):
    """clip_loss_nada.CLIPLoss restated around an image encoder and an E_T(list of strings) callable."""

    def __init__(self, visual, text_encoder, lambda_direction=1.0, lambda_global=0.0, lambda_manifold=0.0,
                 logit_scale=math.log(100.0)):
        super().__init__()
        self.visual = visual
        self.text_encoder = text_encoder
        self.lambda_direction, self.lambda_global, self.lambda_manifold = lambda_direction, lambda_global, lambda_manifold
        self.logit_scale = torch.tensor(logit_scale, dtype=torch.float32)
        self.mean, self.std = get_mean_std()
        self.target_direction = None
        self.src_text_features = None
        self.target_text_features = None

    def get_text_features(self, class_str):
        f = self.text_encoder([t.format(class_str) for t in NADA_TEMPLATES]).detach()
        return f / f.norm(dim=-1, keepdim=True)

    def compute_text_direction(self, source_class, target_class):
        d = (self.get_text_features(target_class) - self.get_text_features(source_class)).mean(0, keepdim=True)
        return d / d.norm(dim=-1, keepdim=True)

    def image_features(self, img):
        f = self.visual(nada_preprocess(img, self.mean, self.std))
        return f / f.norm(dim=-1, keepdim=True)

    def forward(self, src_img, source_class, target_img, target_class):
        loss = 0.0
        if self.lambda_global:
            t = self.text_encoder([f"a {target_class}"]).detach()
            t = t / t.norm(dim=1, keepdim=True)
            logits = self.logit_scale.exp() * self.image_features(target_img) @ t.t()
            loss = loss + self.lambda_global * (1.0 - logits / 100).mean()
        if self.lambda_direction:
            if self.target_direction is None:
                self.target_direction = self.compute_text_direction(source_class, target_class)
            edit = self.image_features(target_img) - self.image_features(src_img)
            edit = edit / edit.norm(dim=-1, keepdim=True)
            loss = loss + self.lambda_direction * (1.0 - F.cosine_similarity(edit, self.target_direction)).mean()
        if self.lambda_manifold:
            if self.src_text_features is None:
                s = self.get_text_features(source_class).mean(0, keepdim=True)
                t = self.get_text_features(target_class).mean(0, keepdim=True)
                self.src_text_features = s / s.norm(dim=-1, keepdim=True)
                self.target_text_features = t / t.norm(dim=-1, keepdim=True)
            cos_text = self.target_text_features @ self.src_text_features.T
            cos_img = (self.image_features(target_img) * self.image_features(src_img)).sum(1).clamp(-1.0, 1.0)
            loss = loss + self.lambda_manifold * (cos_img - cos_text.reshape(())).abs().mean()
        return loss


# ----------------------------------------------------------------------------- IR-SE50


class _SE(nn.Module):
    def __init__(self, c, reduction=16):
        super().__init__()
        self.avg_pool = nn.AdaptiveAvgPool2d(1)
        self.fc1 = nn.Conv2d(c, c // reduction, 1, bias=False)
        self.relu = nn.ReLU(inplace=True)
        self.fc2 = nn.Conv2d(c // reduction, c, 1, bias=False)
        self.sigmoid = nn.Sigmoid()

    def forward(self, x):
        return x * self.sigmoid(self.fc2(self.relu(self.fc1(self.avg_pool(x)))))


class _IRSEUnit(nn.Module):
    def __init__(self, cin, depth, stride):
        super().__init__()
        if cin == depth:
            self.shortcut_layer = nn.MaxPool2d(1, stride)
        else:
            self.shortcut_layer = nn.Sequential(nn.Conv2d(cin, depth, 1, stride, bias=False), nn.BatchNorm2d(depth))
        self.res_layer = nn.Sequential(
            nn.BatchNorm2d(cin), nn.Conv2d(cin, depth, 3, 1, 1, bias=False), nn.PReLU(depth),
            nn.Conv2d(depth, depth, 3, stride, 1, bias=False), nn.BatchNorm2d(depth), _SE(depth, 16))

    def forward(self, x):
        return self.res_layer(x) + self.shortcut_layer(x)


# (in_channels, depth, units) per stage for the 50-layer variant (helpers.py:29-53).
IRSE50_STAGES = [(64, 64, 3), (64, 128, 4), (128, 256, 14), (256, 512, 3)]


class _Flatten(nn.Module):
    def forward(self, x):
        return x.reshape(x.shape[0], -1)


class IRSE50(nn.Module):
    """ArcFace IR-SE50 backbone at 112x112 (model_irse.py:10-49, mode='ir_se')."""

    def __init__(self, drop_ratio=0.6):
        super().__init__()
        self.input_layer = nn.Sequential(nn.Conv2d(3, 64, 3, 1, 1, bias=False), nn.BatchNorm2d(64), nn.PReLU(64))
        units = []
        for cin, depth, n in IRSE50_STAGES:
            units.append(_IRSEUnit(cin, depth, 2))
            units += [_IRSEUnit(depth, depth, 1) for _ in range(n - 1)]
        self.body = nn.Sequential(*units)
        self.output_layer = nn.Sequential(nn.BatchNorm2d(512), nn.Dropout(drop_ratio), _Flatten(),
                                          nn.Linear(512 * 7 * 7, 512), nn.BatchNorm1d(512, affine=True))

    def forward(self, x):
        x = self.output_layer(self.body(self.input_layer(x)))
        return x / torch.norm(x, 2, 1, True)


class IDLoss(nn.Module):
    def __init__(self, facenet):
        super().__init__()
        self.facenet = facenet.eval()

    def extract_feats(self, x):
        if x.shape[2] != 256:
            x = F.adaptive_avg_pool2d(x, (256, 256))
        x = x[:, :, 35:223, 32:220]
        x = F.adaptive_avg_pool2d(x, (112, 112))
        return self.facenet(x)

    def forward(self, y_hat, y):
        y_feats = self.extract_feats(y).detach()
        y_hat_feats = self.extract_feats(y_hat)
        n = y.shape[0]
        loss = 0
        for i in range(n):
            loss = loss + (1 - y_hat_feats[i].dot(y_feats[i]))
        return loss / n, 0.0


def compute_loss(img, original_img, styles, styles2, clip_loss, id_loss, mean, std,
                 identity_loss_coef=0.6, clip_loss_coef=1.0, l2_reg_coef=0.1,
                 trainable=(2, 3, 5, 6, 8, 9, 11, 12), clip_loss2=None, clip_loss_type="default",
                 text_prompt=None, negative_text_prompt=None):
    """find_direction.py:172-200; clip_loss2 = the ViT-B/16 loss of --clip_type double (:163-166: L32 + 0.5 L16).
    clip_loss_type 'nada' / 'nada_global': CLIPLossNADA objects called on the raw images with the prompts as
    classes (:150-157)."""
    identity_loss = id_loss(img, original_img)[0] * identity_loss_coef
    if clip_loss_type in ("nada", "nada_global"):
        clip_alignment_loss = clip_loss(original_img, negative_text_prompt, img, text_prompt)
        if clip_loss2 is not None:
            clip_alignment_loss = clip_alignment_loss + 0.5 * clip_loss2(original_img, negative_text_prompt, img,
                                                                         text_prompt)
    else:
        src, tgt = unprocess(original_img, mean, std), unprocess(img, mean, std)
        clip_alignment_loss = clip_loss(src, tgt)
        if clip_loss2 is not None:
            clip_alignment_loss = clip_alignment_loss + 0.5 * clip_loss2(src, tgt)
    clip_alignment_loss = clip_alignment_loss * clip_loss_coef
    t = list(trainable)
    l2 = l2_reg_coef * F.mse_loss(styles2[:, t], styles[:, t])
    loss = identity_loss + clip_alignment_loss + l2
    return loss, {"clip_loss": clip_alignment_loss, "identity_loss": identity_loss, "landmarks_loss": 0.0,
                  "l2_loss": l2}


_ = math
