"""StyleGAN-NADA CLIP losses (clip_loss_nada.py), the ``--clip_loss_type nada | nada_global`` branch of
find_direction.py:100-114,150-157 and train_latent_mapper.py.

What the reference computes (``CLIPLoss`` of clip_loss_nada.py, third-party ``clip`` for the towers):

* ``preprocess`` (:72-75): torchvision ``Normalize(-1, 2)`` ((x + 1) / 2, GAN output -> [0, 1]), the CLIP
  preprocess' ``Resize(224, BICUBIC)`` + ``CenterCrop(224)``, CLIP ``Normalize`` -- no clamp.  Here one gfx950
  kernel each way (``smc_clip_preprocess_nada_f32`` / ``_bwd_f32``, csrc/unprocess.hip).
* ``get_text_features`` (:126-136): the class string in each of the 27 ``imagenet_templates_small``, encoded,
  each row normalised.  ``compute_text_direction`` (:146-153): mean over templates of (target - source), normalised.
* ``get_image_features`` (:138-144): E_I(preprocess(img)), normalised.
* ``clip_directional_loss`` (:206-218): 1 - cos(norm(f_tgt - f_src), text direction), batch mean.
* ``global_clip_loss`` (:220-229): the CLIP model forward on the target and the single prompt ``"a {target}"``:
  1 - exp(logit_scale) * cos(f_img, f_text) / 100, batch mean.
* ``clip_angle_loss`` (:184-201): L1 between cos(f_tgt, f_src) and cos(t_target, t_source) of the template-mean
  text features (``set_text_features``, :177-182).
* ``forward`` (:324-346): lambda_global * global + lambda_patch * patch + lambda_direction * direction +
  lambda_manifold * manifold (+ lambda_texture * RN50 feature MSE when a texture image is passed).

Not built: the patch terms (``part_templates`` is None in the reference, :11, so ``compose_text_with_templates``
fails there for any lambda_patch != 0) and the texture term (needs ``clip.load("RN50")``, :94, which
find_direction never uses: no texture image is ever passed).  Both raise.

The image tower is the HIP ViT (``vit_hip``, default) or the PyTorch-ROCm one (``impl='torch'``).  Text: the
CLIP text tower + BPE tokenizer (``clip_state_dict`` + ``bpe_path``, stylemc_amd.clip_text), any callable
``text_encoder(list[str]) -> [n, D]`` (un-normalised E_T), or seeded per-string embeddings
(``synthetic_weights=True``, tests / benchmarks only).  The text side runs once per loss object.

``NadaTerms`` is the per-sample form find_direction's DirectionFinder uses (sum-form loss shardable over
ranks; [edited; original] through the tower as one batch, backward for the edited half).
"""
import math

import torch
import torch.nn.functional as F
from torch import nn

from . import _hip, clip_model, synthetic, vit_hip
from .clip_loss import MODEL_NAMES, split_clip_state_dict

# clip_loss_nada.py:12-40 (the prompt templates are data the direction depends on)
imagenet_templates_small = [
    'a photo of a {}.', 'a rendering of a {}.', 'a cropped photo of the {}.', 'the photo of a {}.',
    'a photo of a clean {}.', 'a photo of a dirty {}.', 'a dark photo of the {}.', 'a photo of my {}.',
    'a photo of the cool {}.', 'a close-up photo of a {}.', 'a bright photo of the {}.', 'a cropped photo of a {}.',
    'a photo of the {}.', 'a good photo of the {}.', 'a photo of one {}.', 'a close-up photo of the {}.',
    'a rendition of the {}.', 'a photo of the clean {}.', 'a rendition of a {}.', 'a photo of a nice {}.',
    'a good photo of a {}.', 'a photo of the nice {}.', 'a photo of the small {}.', 'a photo of the weird {}.',
    'a photo of the large {}.', 'a photo of a cool {}.', 'a photo of a small {}.',
]
part_templates = None   # clip_loss_nada.py:11

CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)


class NadaPreprocessFn(torch.autograd.Function):
    """clip_loss_nada.py:72-75 preprocess for square fp32 GPU images: one gfx950 kernel each way."""

    @staticmethod
    def forward(ctx, img, mean, std, size):
        img = img.contiguous()
        n, c, h, w = img.shape
        y = torch.empty(n, c, size, size, device=img.device, dtype=torch.float32)
        _hip.call("smc_clip_preprocess_nada_f32", img.data_ptr(), n, c, h, w, size, size, mean.data_ptr(),
                  std.data_ptr(), y.data_ptr(), _hip.stream())
        ctx.save_for_backward(img, mean, std)
        ctx.size = size
        return y

    @staticmethod
    def backward(ctx, gy):
        img, mean, std = ctx.saved_tensors
        n, c, h, w = img.shape
        gy = gy.contiguous()
        dimg = torch.empty_like(img)
        _hip.call("smc_clip_preprocess_nada_bwd_f32", img.data_ptr(), gy.data_ptr(), n, c, h, w, ctx.size, ctx.size,
                  mean.data_ptr(), std.data_ptr(), dimg.data_ptr(), _hip.stream())
        return dimg, None, None, None


def nada_preprocess(img, mean, std, size=224):
    """(img + 1) / 2 -> bicubic Resize(size) + CenterCrop(size) -> (x - mean) / std (no clamp)."""
    if not (img.is_cuda and img.dtype == torch.float32 and img.ndim == 4 and img.shape[2] == img.shape[3]
            and img.shape[2] >= size):
        raise RuntimeError(f"NADA preprocess: square fp32 GPU images of >= {size} px only (got {tuple(img.shape)}, "
                           f"{img.device}); the HIP kernel is the only implementation")
    return NadaPreprocessFn.apply(img, mean.reshape(-1).contiguous(), std.reshape(-1).contiguous(), size)


class DirectionLoss(nn.Module):
    """clip_loss_nada.py:43-59: 'cosine' -> 1 - cos, 'mse' / 'mae' -> the plain losses."""

    def __init__(self, loss_type="mse"):
        super().__init__()
        if loss_type not in ("mse", "cosine", "mae"):
            raise KeyError(loss_type)
        self.loss_type = loss_type

    def forward(self, x, y):
        if self.loss_type == "cosine":
            return 1.0 - F.cosine_similarity(x, y)
        return F.mse_loss(x, y) if self.loss_type == "mse" else F.l1_loss(x, y)


def _text_encoder_from_state_dict(text_sd, bpe_path, device, impl):
    from . import clip_text
    tower = clip_text.TextTransformer.from_state_dict(text_sd).eval().requires_grad_(False).to(device)
    tok = clip_text.SimpleTokenizer(bpe_path)
    return lambda strings: tower.encode_text(tok.tokenize(list(strings)), impl=impl)


class CLIPLoss(nn.Module):
    """clip_loss_nada.CLIPLoss with the reference's constructor arguments; weight sources as in
    stylemc_amd.clip_loss.CLIPLoss (no ``clip.load`` offline).  ``logit_scale``: the CLIP model's parameter
    (state_dict key ``logit_scale``; ln 100 for synthetic weights, the value the released models carry)."""

    takes_raw_images = True

    def __init__(self, device="cuda", lambda_direction=1., lambda_patch=0., lambda_global=0., lambda_manifold=0.,
                 lambda_texture=0., patch_loss_type="mae", direction_loss_type="cosine", clip_model="ViT-B/32",
                 clip_state_dict=None, visual_state_dict=None, text_encoder=None, bpe_path=None, logit_scale=None,
                 impl="hip", synthetic_weights=False, seed=4, text_seed=0, visual=None):
        super().__init__()
        name = MODEL_NAMES.get(clip_model, clip_model)
        if name not in clip_model_configs():
            raise ValueError(f"clip_model must be ViT-B/32 or ViT-B/16, got {clip_model!r}")
        if lambda_patch:
            raise NotImplementedError("lambda_patch: part_templates is None in the reference (clip_loss_nada.py:11), "
                                      "so its patch terms cannot run there either")
        self.device = torch.device(device)
        self.model_name = name
        text_sd = None
        if clip_state_dict is not None:
            visual_state_dict, text_sd = split_clip_state_dict(clip_state_dict)
            if logit_scale is None and "logit_scale" in clip_state_dict:
                logit_scale = float(torch.as_tensor(clip_state_dict["logit_scale"]).float())
        if visual is None:
            if visual_state_dict is None and not synthetic_weights:
                raise ValueError(f"CLIPLoss NADA ({name}): no image-tower weights (clip_state_dict / "
                                 f"visual_state_dict); synthetic_weights=True selects seeded weights explicitly")
            builder = vit_hip.build_visual if impl == "hip" else clip_model.build_visual
            visual = builder(name, visual_state_dict, seed=seed, device=self.device)
        self.visual = visual
        if text_encoder is None:
            if text_sd is not None and bpe_path is not None and "ln_final.weight" in text_sd:
                text_encoder = _text_encoder_from_state_dict(text_sd, bpe_path, self.device, impl)
            elif synthetic_weights:
                text_encoder = lambda strings: synthetic.text_embeddings(strings, seed=text_seed)  # noqa: E731
            else:
                raise ValueError(f"CLIPLoss NADA ({name}): no text encoder -- give a CLIP state_dict with its text "
                                 f"tower plus the BPE merges file (bpe_path), or text_encoder=")
        self.text_encoder = text_encoder
        self.logit_scale = math.log(100.0) if logit_scale is None else float(logit_scale)
        # logit_scale.exp() of the CLIP forward, in fp32 as the parameter is stored
        self.logit_scale_exp = float(torch.tensor(self.logit_scale, dtype=torch.float32).exp())
        mean = torch.tensor(CLIP_MEAN, dtype=torch.float32, device=self.device)
        std = torch.tensor(CLIP_STD, dtype=torch.float32, device=self.device)
        self.register_buffer("mean", mean, persistent=False)
        self.register_buffer("std", std, persistent=False)
        self.target_direction = None
        self.src_text_features = None
        self.target_text_features = None
        self._global_text = {}
        self.direction_loss = DirectionLoss(direction_loss_type)
        self.patch_loss = DirectionLoss(patch_loss_type)
        self.lambda_global = lambda_global
        self.lambda_patch = lambda_patch
        self.lambda_direction = lambda_direction
        self.lambda_manifold = lambda_manifold
        self.lambda_texture = lambda_texture

    # ---- text side (once per loss object)
    def encode_text(self, strings):
        with torch.no_grad():
            return torch.as_tensor(self.text_encoder(list(strings))).to(self.device, torch.float32)

    @staticmethod
    def compose_text_with_templates(text, templates=imagenet_templates_small):
        return [template.format(text) for template in templates]

    def get_text_features(self, class_str, templates=imagenet_templates_small, norm=True):
        f = self.encode_text(self.compose_text_with_templates(class_str, templates))
        return f / f.norm(dim=-1, keepdim=True) if norm else f

    def compute_text_direction(self, source_class, target_class):
        d = (self.get_text_features(target_class) - self.get_text_features(source_class)).mean(dim=0, keepdim=True)
        return d / d.norm(dim=-1, keepdim=True)

    def set_text_features(self, source_class, target_class):
        s = self.get_text_features(source_class).mean(dim=0, keepdim=True)
        self.src_text_features = s / s.norm(dim=-1, keepdim=True)
        t = self.get_text_features(target_class).mean(dim=0, keepdim=True)
        self.target_text_features = t / t.norm(dim=-1, keepdim=True)

    def global_text_features(self, text):
        """The normalised E_T of the global loss' prompt list (CLIP model forward, :227)."""
        key = tuple(text)
        if key not in self._global_text:
            f = self.encode_text(list(text))
            self._global_text[key] = f / f.norm(dim=-1, keepdim=True)
        return self._global_text[key]

    def prepare(self, source_class, target_class):
        """Every text-side quantity forward() will need, computed once (the reference does it lazily)."""
        if self.lambda_direction and self.target_direction is None:
            self.target_direction = self.compute_text_direction(source_class, target_class)
        if self.lambda_manifold and self.src_text_features is None:
            self.set_text_features(source_class, target_class)
        if self.lambda_global:
            self.global_text_features([f"a {target_class}"])

    # ---- image side
    def encode_images(self, images, n_grad=None):
        x = nada_preprocess(images, self.mean, self.std, self.visual.input_resolution)
        if n_grad is not None and getattr(self.visual, "supports_partial_grad", False):
            return self.visual(x, n_grad=n_grad)
        return self.visual(x)

    def get_image_features(self, img, norm=True):
        f = self.encode_images(img)
        return f / f.norm(dim=-1, keepdim=True) if norm else f

    def per_sample_terms(self, f_tgt, f_src, source_class, target_class):
        """Per-image loss of normalised image features (f_src may be None when no term needs it): sum over the
        enabled terms of lambda * term_i, whose batch mean is forward()."""
        self.prepare(source_class, target_class)
        out = 0.0
        if self.lambda_global:
            t = self.global_text_features([f"a {target_class}"])
            logits = self.logit_scale_exp * f_tgt @ t.t()                            # [N, 1]
            out = out + self.lambda_global * (1.0 - logits / 100).mean(dim=1)
        if self.lambda_direction:
            edit = f_tgt - f_src
            edit = edit / edit.norm(dim=-1, keepdim=True)
            out = out + self.lambda_direction * self.direction_loss(edit, self.target_direction)
        if self.lambda_manifold:
            cos_text = (self.target_text_features @ self.src_text_features.t()).reshape(())
            cos_img = (f_tgt * f_src).sum(dim=1).clamp(-1.0, 1.0)
            out = out + self.lambda_manifold * (cos_img - cos_text).abs()
        return out

    def needs_source(self):
        return bool(self.lambda_direction or self.lambda_manifold)

    def forward(self, src_img, source_class, target_img, target_class, texture_image=None):
        if self.lambda_texture and texture_image is not None:
            raise NotImplementedError("lambda_texture: the RN50 feature loss (clip_loss_nada.py:318-322) is not built")
        f_tgt = self.get_image_features(target_img)
        f_src = self.get_image_features(src_img) if self.needs_source() else None
        return self.per_sample_terms(f_tgt, f_src, source_class, target_class).mean()


def clip_model_configs():
    return clip_model.VIT_CONFIGS


class NadaTerms(nn.Module):
    """A NADA CLIPLoss with its (source, target) classes bound, in the per-sample interface of
    DirectionFinder (find_direction.py:150-157: clip_loss(original_img, negative_text_prompt, gen_img,
    text_prompt)).  Inputs are the raw generator images (the loss preprocesses them itself)."""

    takes_raw_images = True

    def __init__(self, loss, source_class, target_class):
        super().__init__()
        self.loss = loss
        self.source_class, self.target_class = source_class, target_class
        loss.prepare(source_class, target_class)

    @torch.no_grad()
    def encode_src(self, src_image):
        return self.loss.get_image_features(src_image) if self.loss.needs_source() else None

    def per_sample_with(self, src_feats, tgt_image):
        return self.loss.per_sample_terms(self.loss.get_image_features(tgt_image), src_feats, self.source_class,
                                          self.target_class)

    def per_sample_pair(self, tgt_image, src_image):
        n = tgt_image.shape[0]
        if not self.loss.needs_source():
            return self.per_sample_with(None, tgt_image)
        f = self.loss.encode_images(torch.cat([tgt_image, src_image.detach()]), n_grad=n)
        f = f / f.norm(dim=-1, keepdim=True)
        return self.loss.per_sample_terms(f[:n], f[n:].detach(), self.source_class, self.target_class)

    def per_sample(self, src_image, tgt_image):
        return self.per_sample_with(self.encode_src(src_image), tgt_image)

    def forward(self, src_image, tgt_image):
        return self.per_sample(src_image, tgt_image).mean()
