"""Directional CLIP loss (clip_loss.py:7-34): mean(1 - cos(norm(E(tgt) - E(src)), norm(T+ - T-))).

Without the third-party ``clip`` package and its weights (absent offline) the text direction is either
given (``text_features``) or a seeded unit vector derived from the two prompts
(``synthetic.text_direction``).  The image tower is ``vit_hip.HipVisionTransformer`` (``impl='hip'``,
the default: the whole ViT on the gfx950 kernel library, BASELINE config 4) or
``clip_model.VisionTransformer`` (``impl='torch'``: PyTorch-ROCm ops, BASELINE config 2).
``per_sample`` returns 1 - cos_i so the loss can be sharded over ranks and summed.
"""
import torch
import torch.nn.functional as F
from torch import nn

from . import clip_model, synthetic, vit_hip


class CLIPLoss(nn.Module):
    def __init__(self, device="cuda", text_prompt="", negative_text_prompt="", clip_type="small", visual=None,
                 text_features=None, visual_state_dict=None, seed=4, impl="hip"):
        super().__init__()
        name = "ViT-B/32" if clip_type == "small" else "ViT-B/16"
        self.model_name = name
        if impl not in ("hip", "torch"):
            raise ValueError(f"impl must be 'hip' or 'torch', got {impl!r}")
        builder = vit_hip.build_visual if impl == "hip" else clip_model.build_visual
        self.visual = visual if visual is not None else builder(name, visual_state_dict, seed=seed, device=device)
        if text_features is None:
            text_features = synthetic.text_direction(text_prompt, negative_text_prompt)
        t = torch.as_tensor(text_features, dtype=torch.float32).reshape(1, -1).to(device)
        self.register_buffer("text_features", t / t.norm(dim=1, keepdim=True))

    def encode_image(self, image):
        return self.visual(image)

    @torch.no_grad()
    def encode_src(self, src_image):
        """E(src): the original image's embedding (no gradient flows to it in the reference)."""
        return self.visual(src_image)

    def per_sample_with(self, src_emb, tgt_image):
        f = self.visual(tgt_image) - src_emb
        f = f / f.norm(dim=1, keepdim=True)
        return 1 - F.cosine_similarity(f, self.text_features)

    def per_sample_pair(self, tgt_image, src_image):
        """per_sample(src, tgt) with both images in ONE tower batch [tgt; src]: the backward runs for the
        tgt half only (E(src) carries no gradient in the reference)."""
        n = tgt_image.shape[0]
        x = torch.cat([tgt_image, src_image.detach()])
        e = self.visual(x, n_grad=n) if getattr(self.visual, "supports_partial_grad", False) else self.visual(x)
        f = e[:n] - e[n:].detach()
        f = f / f.norm(dim=1, keepdim=True)
        return 1 - F.cosine_similarity(f, self.text_features)

    def per_sample(self, src_image, tgt_image):
        return self.per_sample_with(self.encode_src(src_image), tgt_image)

    def forward(self, src_image, tgt_image):
        return self.per_sample(src_image, tgt_image).mean()
