"""Directional CLIP loss (clip_loss.py:7-34): mean(1 - cos(norm(E(tgt) - E(src)), norm(T+ - T-))).

The reference gets both CLIP towers from the third-party ``clip.load`` (clip_loss.py:11-13) and encodes the
two prompts once (:15-18).  Offline there is no ``clip`` package and no weights, so the weights come from
the caller:

* ``clip_state_dict``: an OpenAI CLIP model state_dict (``visual.*`` + the text keys; e.g. saved with
  ``torch.save(clip.load(name, jit=False)[0].state_dict())``).  Its visual half drives the image tower, and
  with a BPE merges file (``bpe_path``, the clip package's ``bpe_simple_vocab_16e6.txt.gz``) its text half
  computes ``text_features`` exactly as :15-18 (stylemc_amd.clip_text).
* ``visual_state_dict`` / ``text_features``: the image tower's ``visual.*`` weights and/or precomputed
  ``norm(E_T(pos) - E_T(neg))``.
* ``synthetic=True``: seeded synthetic weights and a prompt-hash text direction -- benchmarks and tests
  only; never chosen implicitly (a missing weight source raises, like ``clip.load`` would).

The image tower is ``vit_hip.HipVisionTransformer`` (``impl='hip'``, the default: the whole ViT on the
gfx950 kernel library, BASELINE config 4) or ``clip_model.VisionTransformer`` (``impl='torch'``:
PyTorch-ROCm ops, BASELINE config 2).  ``per_sample`` returns 1 - cos_i so the loss can be sharded over
ranks and summed.
"""
import torch
import torch.nn.functional as F
from torch import nn

from . import clip_model, rowops, synthetic, vit_hip

MODEL_NAMES = {"small": "ViT-B/32", "large": "ViT-B/16"}

# The loss head as one autograd node whose gradient is formed in the forward pass (module switch for A/B): autograd's
# graph of the head (difference, norm, division, cosine_similarity, 1 - x) replays ~28 small kernels in the backward
# on the step's critical path, between the CLIP forward and its backward; here the backward is one multiply.
FUSED_HEAD = True


class _DirectionHead(torch.autograd.Function):
    """1 - cos(normalize(e - src), t) per sample, t unit-norm.  Forward: the reference's ops (same values).  Backward:
    d/de = (cos u - t) / |e - src| per sample with u = normalize(e - src) -- the exact gradient of the formula up to
    |u| = |t| = 1 (each within a few ulp in fp32), against autograd through cosine_similarity's own normalisation."""

    @staticmethod
    def forward(ctx, e, src, t):
        if e.is_cuda:   # one gfx950 launch, rows reduced in a fixed order (batch-invariant, rowops)
            loss, gf = rowops.direction_head(e, src, t)
            ctx.save_for_backward(gf)
            return loss
        f = e - src
        nf = f.norm(dim=1, keepdim=True)
        u = f / nf
        cos = F.cosine_similarity(u, t)
        ctx.save_for_backward(torch.addcmul(-t, cos[:, None], u) / nf)
        return 1 - cos

    @staticmethod
    def backward(ctx, g):
        (gf,) = ctx.saved_tensors
        return g[:, None] * gf, None, None


def direction_loss(e, src, t):
    if FUSED_HEAD and e.requires_grad and not src.requires_grad and not t.requires_grad:
        return _DirectionHead.apply(e, src, t)
    f = e - src
    f = f / f.norm(dim=1, keepdim=True)
    return 1 - F.cosine_similarity(f, t)


def split_clip_state_dict(sd):
    """OpenAI CLIP model state_dict -> (visual state_dict without the 'visual.' prefix, text state_dict)."""
    visual = {k[len("visual."):]: v for k, v in sd.items() if k.startswith("visual.")}
    text = {k: v for k, v in sd.items() if not k.startswith("visual.") and k not in ("logit_scale",)}
    return visual, text


class CLIPLoss(nn.Module):
    def __init__(self, device="cuda", text_prompt="", negative_text_prompt="", clip_type="small", visual=None,
                 text_features=None, visual_state_dict=None, clip_state_dict=None, bpe_path=None, seed=4,
                 impl="hip", synthetic_weights=False):
        super().__init__()
        name = MODEL_NAMES.get(clip_type, clip_type)
        if name not in clip_model.VIT_CONFIGS:
            raise ValueError(f"clip_type must be 'small' (ViT-B/32) or 'large' (ViT-B/16), got {clip_type!r}")
        self.model_name = name
        if impl not in ("hip", "torch"):
            raise ValueError(f"impl must be 'hip' or 'torch', got {impl!r}")
        text_sd = None
        if clip_state_dict is not None:
            visual_state_dict, text_sd = split_clip_state_dict(clip_state_dict)
        if visual is None:
            if visual_state_dict is None and not synthetic_weights:
                raise ValueError(f"CLIPLoss({name}): no image-tower weights (clip_state_dict / visual_state_dict); "
                                 f"synthetic_weights=True selects seeded synthetic weights explicitly")
            builder = vit_hip.build_visual if impl == "hip" else clip_model.build_visual
            visual = builder(name, visual_state_dict, seed=seed, device=device)
        self.visual = visual
        if text_features is None:
            if text_sd is not None and bpe_path is not None and "ln_final.weight" in text_sd:
                from . import clip_text
                tower = clip_text.TextTransformer.from_state_dict(text_sd).eval().requires_grad_(False).to(device)
                tok = clip_text.SimpleTokenizer(bpe_path)
                text_features = clip_text.text_direction(tower, tok, text_prompt, negative_text_prompt, impl=impl)
            elif synthetic_weights:
                text_features = synthetic.text_direction(text_prompt, negative_text_prompt)
            else:
                raise ValueError(f"CLIPLoss({name}): no text direction -- give text_features, or a CLIP state_dict "
                                 f"with its text tower plus the BPE merges file (bpe_path)")
        t = torch.as_tensor(text_features, dtype=torch.float32).reshape(1, -1).to(device)
        self.register_buffer("text_features", t / t.norm(dim=1, keepdim=True))

    def encode_image(self, image):
        return self.visual(image)

    @torch.no_grad()
    def encode_src(self, src_image):
        """E(src): the original image's embedding (no gradient flows to it in the reference)."""
        return self.visual(src_image)

    def per_sample_with(self, src_emb, tgt_image):
        return direction_loss(self.visual(tgt_image), src_emb, self.text_features)

    def per_sample_pair(self, tgt_image, src_image):
        """per_sample(src, tgt) with both images in ONE tower batch [tgt; src]: the backward runs for the
        tgt half only (E(src) carries no gradient in the reference)."""
        n = tgt_image.shape[0]
        x = torch.cat([tgt_image, src_image.detach()])
        e = self.visual(x, n_grad=n) if getattr(self.visual, "supports_partial_grad", False) else self.visual(x)
        return direction_loss(e[:n], e[n:].detach(), self.text_features)

    def per_sample(self, src_image, tgt_image):
        return self.per_sample_with(self.encode_src(src_image), tgt_image)

    def forward(self, src_image, tgt_image):
        return self.per_sample(src_image, tgt_image).mean()
