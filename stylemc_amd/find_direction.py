"""find_direction on MI355X: drop-in for the reference's find_direction.py (CLI flags kept).

The optimisation (find_direction.py:259-351) is restated with its intended behaviour:
  * lr_t = 0.5*lr0*(1 + cos(pi*t/T)), T = n_epochs*ceil(n/B)                        (:297-301)
  * batch index i = randint(0, ceil(n/B)) with replacement (seeded here; unseeded in :303)
  * styles2 = styles + direction on rows T = [2,3,5,6,8,9,11,12]                  (:307-308)
  * loss = id_c*ID(img, orig) + clip_c*CLIP(orig, img) + l2_c*mse(styles2[:,T], styles[:,T])  (:172-200)
  * SGD p -= lr_t * grad                                                             (:336-339)
  * output npz key 's' [1,26,512]: ``styles_direction`` as the reference saves it -- the delta written
    into it at the start of the last iteration (:307, :349-351)
Start point: the reference starts from delta = 0 (:270-273), where img == original_img bit for bit and
the directional CLIP loss normalises a zero feature difference (clip_loss.py:29-30): 0/0 = NaN, which
then poisons every later step.  Runs therefore start from ``initial_delta(seed, init_std)``, a seeded
N(0, init_std) direction (--init_std 0 reproduces the literal zero start).
Landmarks: the reference computes that term under torch.no_grad (:90), so it never changes the
direction; a non-zero --landmarks_loss_coef is accepted and ignored with a warning.
generate_image is called with the missing ``device`` fixed (:309,312 raise TypeError as shipped).

Multi-GPU: every rank draws the same i, takes its contiguous slice of the global batch and returns one row per
image (its gradient and loss terms); one all_gather of those rows (World.gather_rows) and one fixed-order sum over the
global batch (combine) give every rank the same buffer, bit-equal to the single-process one (stylemc_amd.dist).
"""
import contextlib
import math
import os
import time
import warnings

import numpy as np
import torch
import torch.nn.functional as F

from . import _hip
from . import dist as _dist
from . import rowops, utils

N_STYLE_CHANNELS = utils.N_STYLE_CHANNELS
S_TRAINABLE_SPACE_CHANNELS = utils.S_TRAINABLE_SPACE_CHANNELS
S_NON_TRAINABLE_SPACE_CHANNELS = utils.S_NON_TRAINABLE_SPACE_CHANNELS
RESOLUTION_DICT = {256: 6, 512: 7, 1024: 8}


class UnprocessFn(torch.autograd.Function):
    """unprocess() for square fp32 GPU images downsampled to `size`: one gfx950 kernel each way
    (smc_clip_unprocess_f32 / _bwd_f32, csrc/unprocess.hip)."""

    @staticmethod
    def forward(ctx, img, mean, std, size):
        from . import _hip
        img = img.contiguous()
        n, c, h, w = img.shape
        mean = mean.reshape(-1).contiguous()
        std = std.reshape(-1).contiguous()
        y = torch.empty(n, c, size, size, device=img.device, dtype=torch.float32)
        _hip.call("smc_clip_unprocess_f32", _hip.ptr(img), n, c, h, w, size, size, _hip.ptr(mean), _hip.ptr(std),
                  y.data_ptr(), _hip.stream())
        ctx.save_for_backward(img, mean, std)
        ctx.size = size
        return y

    @staticmethod
    def backward(ctx, gy):
        from . import _hip
        img, mean, std = ctx.saved_tensors
        n, c, h, w = img.shape
        gy = gy.contiguous()
        dimg = torch.empty_like(img)
        _hip.call("smc_clip_unprocess_bwd_f32", _hip.ptr(img), _hip.ptr(gy), n, c, h, w, ctx.size, ctx.size,
                  _hip.ptr(mean), _hip.ptr(std), dimg.data_ptr(), _hip.stream())
        return dimg, None, None, None


def unprocess(img, mean, std, size=224):
    """find_direction.py:49-52 with torchvision-0.8 tensor Resize(224, BICUBIC) + CenterCrop(224)."""
    if (img.is_cuda and img.dtype == torch.float32 and img.ndim == 4 and img.shape[2] == img.shape[3]
            and img.shape[2] >= size and mean.numel() == img.shape[1]):
        return UnprocessFn.apply(img, mean, std, size)
    x = (img * 127.5 + 128).clamp(0, 255)
    h, w = x.shape[-2:]
    nh, nw = (size, int(size * w / h)) if h <= w else (int(size * h / w), size)
    x = F.interpolate(x, size=(nh, nw), mode="bicubic", align_corners=False)
    top, left = int(round((nh - size) / 2.0)), int(round((nw - size) / 2.0))
    x = x[..., top:top + size, left:left + size]
    return (x / 255 - mean) / std


def compute_loss(img, original_img, transf, mean, std, device, clip_loss_type, clip_type, clip_loss_coef,
                 clip_loss1_func, clip_loss2_func, text_prompt, negative_text_prompt, id_loss, identity_loss_coef,
                 landmarks_loss, landmarks_loss_coef, mobilenet, img_size, styles, styles2, l2_reg_coef):
    """find_direction.py:172-200 with the reference's signature (unbatched form: each loss network sees the
    edited and the original image separately; DirectionFinder.step runs the batched equivalent).

    ``transf`` must be None: the torchvision Resize(224, BICUBIC) + CenterCrop of :258 is built into
    ``unprocess``.  The landmarks term is 0 (computed under no_grad in the reference, :90).  clip_loss_type
    'nada' / 'nada_global': the loss functions are stylemc_amd.clip_loss_nada.CLIPLoss objects, called on the raw
    images with the prompts as classes (compute_clip_loss, :150-157).
    """
    if transf is not None:
        raise ValueError("transf: the bicubic Resize + CenterCrop is built into unprocess(); pass None")
    if clip_loss_type not in ("default", "nada", "nada_global"):
        raise ValueError(f"clip_loss_type must be default, nada or nada_global, got {clip_loss_type!r}")
    identity_loss = id_loss(img, original_img)[0] * identity_loss_coef
    if clip_loss_type != "default":
        clip_alignment_loss = clip_loss1_func(original_img, negative_text_prompt, img, text_prompt)
        if clip_type == "double":
            clip_alignment_loss = clip_alignment_loss + 0.5 * clip_loss2_func(original_img, negative_text_prompt, img,
                                                                              text_prompt)
    else:
        tgt = unprocess(img, mean, std, img_size)
        src = unprocess(original_img, mean, std, img_size)
        clip_alignment_loss = clip_loss1_func(src, tgt)
        if clip_type == "double":
            clip_alignment_loss = clip_alignment_loss + 0.5 * clip_loss2_func(src, tgt)
    clip_alignment_loss = clip_loss_coef * clip_alignment_loss
    T = S_TRAINABLE_SPACE_CHANNELS
    l2 = l2_reg_coef * F.mse_loss(styles2[:, T], styles[:, T])
    loss = identity_loss + clip_alignment_loss + l2
    return loss, {"clip_loss": clip_alignment_loss, "identity_loss": identity_loss, "landmarks_loss": 0.0,
                  "l2_loss": l2}


def initial_delta(seed=0, init_std=0.01, device="cpu"):
    """Seeded starting direction [1, 8, 512] (see the module docstring: an exact zero start is NaN)."""
    g = torch.Generator().manual_seed(int(seed) + 7919)
    return (torch.randn(1, len(S_TRAINABLE_SPACE_CHANNELS), 512, generator=g) * init_std).to(device)


def cosine_lr(lr0, it, total):
    return float(np.cos(np.pi * it / total) * lr0 * 0.5 + lr0 * 0.5)


# The original image's CLIP embeddings computed on the prefetch stream too (CLIP on the critical path then runs the
# edited half only: forward 4 + backward 4 instead of forward 8 + backward 4).  Module switch for A/B:
# off -- measured slower again in round 6, 465.5-468.1 against 472.8-475.6 images/s over three interleaved rounds
# (profiles/r06/prefetch_clip_ab/; round 3: profiles/r03_clip_prefetch_ab.txt).
PREFETCH_CLIP = False

# The loss composition (find_direction.py:318-330: coefficients x batch sums + the l2 term) as one autograd node with
# an analytic backward (module switch for A/B): autograd's graph of those scalar ops replays ~20 tiny kernels between
# the loss heads and the networks' backward, on the step's critical path.
FUSED_TOTAL = True


class _LossTotal(torch.autograd.Function):
    """Forward: the reference's composition op for op (same values); returns (total, parts = [clip, id, 0, l2]).
    Backward: d total / d id_terms = c_id / denom, d / d clip_terms = c_clip / denom and
    d / d d = 2 ((sT + d) - sT) c_l2 / l2_den -- the derivative autograd forms, in one multiply each."""

    @staticmethod
    def forward(ctx, id_terms, clip_terms, d, sT, c_id, c_clip, c_l2, l2_den, denom):
        diff = (sT + d) - sT
        l2_sum = diff.square().sum()
        id_part = c_id * id_terms.sum() / denom
        clip_part = c_clip * clip_terms.sum() / denom
        l2_part = c_l2 * l2_sum / l2_den
        parts = torch.stack([clip_part, id_part, torch.zeros_like(l2_part), l2_part])
        ctx.mark_non_differentiable(parts)
        ctx.save_for_backward(diff)
        ctx.k = (c_id / denom, c_clip / denom, 2.0 * c_l2 / l2_den)
        ctx.shapes = (id_terms.shape, clip_terms.shape)
        return id_part + clip_part + l2_part, parts

    @staticmethod
    def backward(ctx, g, _gparts):
        (diff,) = ctx.saved_tensors
        k_id, k_clip, k_l2 = ctx.k
        gid = (g * k_id).expand(ctx.shapes[0]) if ctx.needs_input_grad[0] else None
        gclip = (g * k_clip).expand(ctx.shapes[1]) if ctx.needs_input_grad[1] else None
        gd = diff * (g * k_l2) if ctx.needs_input_grad[2] else None
        return gid, gclip, gd, None, None, None, None, None, None


class DirectionFinder:
    """State of one find_direction run; ``step()`` is one iteration of the reference's hot loop."""

    def __init__(self, G, styles_array, clip_losses, id_loss, resolution=1024, batch_size=4, learning_rate=1.5,
                 n_epochs=4, identity_loss_coef=0.6, l2_reg_coef=0.1, clip_loss_coef=1.0, noise_mode="const",
                 seed=0, world=None, global_batch=None, temp_shapes=None, init_delta=None, synth_fn=None,
                 overlap=True, batch_losses=True, prefetch_orig=True, stream_factory=None, G2=None, temp_shapes2=None,
                 prefetch_id=True, plan_batch=None, prefetch_clip=None):
        self.G = G
        # the edited image's generator (train_latent_mapper.py:100-106,159-162 --network2; default G itself)
        self.G_edit = G2 if G2 is not None else G
        # how the side / prefetch streams are made (default: torch's stream pool); tools/stream_ab.py A/Bs it
        self.stream_factory = stream_factory or (lambda dev: torch.cuda.Stream(device=dev))
        self.synth_fn = synth_fn or utils.generate_image_rows   # (G, until_k, styles, shapes, noise, delta=)
        self.overlap = overlap                                  # original-image branch on a second stream
        # software pipelining across iterations: the NEXT iteration's original-image synthesis (it depends only
        # on the S codes of the next batch, not on the direction) runs on a third stream during this
        # iteration's backward; every iteration still synthesises its own original image exactly once
        self.prefetch_orig = prefetch_orig
        # ... and that image's IR-SE50 features (no gradient): IR-SE50 is the loss network that bounds the step
        # (tools/sensitivity.py: dropping it saves 1.8 ms, dropping CLIP nothing), so its critical-path share is
        # cut to the edited images' forward + backward; CLIP keeps the [edited; original] batch
        self.prefetch_id = prefetch_id
        self.prefetch_clip = PREFETCH_CLIP if prefetch_clip is None else prefetch_clip
        # Measured and removed (round 4): the original image's CLIP embeddings prefetched too (19.87-20.01 against
        # 19.58-19.71 ms / step, profiles/r03_clip_prefetch_ab.txt), the prefetch replayed as a captured HIP graph
        # (0.7 ms / step slower, profiles/r03_graph_prefetch_ab.txt), the prefetch started after the loss networks'
        # forward or as soon as enqueued instead of after the edited forward (19.46 / 19.05-19.17 against
        # 18.83-18.87 ms, profiles/r03_prefetch_start_ab.txt).  The prefetch starts after this iteration's edited
        # forward (the _fwd_done event).
        self._next_i = None
        self._pref = None
        # edited + original image through each loss network as ONE batch (backward for the edited half)
        self.batch_losses = batch_losses and hasattr(id_loss, "per_sample_pair") and all(
            hasattr(cl, "per_sample_pair") for cl, _ in clip_losses)
        self.device = styles_array.device
        self.styles_array = styles_array
        self.clip_losses = clip_losses            # [(CLIPLoss, weight)], 'double' -> [(B/32, 1), (B/16, .5)]
        self.id_loss = id_loss
        self.until_k = RESOLUTION_DICT.get(resolution, int(math.log2(resolution)) - 2)
        self.B = int(global_batch or batch_size)
        # batch-invariant kernel plans: every launch of a step is planned as for `plan_batch` images (default: the
        # per-rank batch_size) whatever this rank's shard holds, so a shard computes each image's gradient row bit
        # for bit as the whole batch does in one process (smc_set_plan_batch); the rows are then summed in one
        # fixed order over the global batch (combine) -- the N-rank direction equals the 1-rank one exactly
        self.plan_batch = int(plan_batch or batch_size)
        self.lr0 = learning_rate
        self.n_epochs = n_epochs
        self.coef = dict(id=identity_loss_coef, l2=l2_reg_coef, clip=clip_loss_coef)
        self.noise_mode = noise_mode
        self.world = world or _dist.World()
        self.temp_shapes = temp_shapes if temp_shapes is not None else utils.get_temp_shapes(G)
        self.temp_shapes_edit = self.temp_shapes if G2 is None else (
            temp_shapes2 if temp_shapes2 is not None else utils.get_temp_shapes(G2))
        self.n_items = styles_array.shape[0]
        self.num_batches = math.ceil(self.n_items / self.B)
        self.total_iterations = self.num_batches * n_epochs
        self.rng = np.random.RandomState(seed)
        self.it = 0
        T = S_TRAINABLE_SPACE_CHANNELS
        self.styles_direction = torch.zeros(1, N_STYLE_CHANNELS, 512, device=self.device)
        # device-resident row index: indexing with the Python list would copy a host index tensor to the
        # GPU on every use, a blocking copy that drains the stream mid-step
        self.t_idx = torch.tensor(T, dtype=torch.long, device=self.device)
        self.delta = self.styles_direction[:, T].clone()
        self._offset = None
        if init_delta is not None:
            self.delta = init_delta.detach().to(self.device, torch.float32).reshape(1, len(T), 512).clone()
        self.mean, self.std = utils.get_mean_std(self.device)
        self.images_per_step = 2 * self.B          # edited + original per seed
        self.last = None

    def load_direction(self, direction):
        """--resume: start from a saved [1, 26, 512] direction (the reference's :266-271, with its
        ``map_location`` TypeError fixed).  The reference adds the WHOLE styles_direction to the styles
        (styles2 = styles + styles_direction, :307-308) and trains only the T rows, so any non-zero non-T rows
        of the resumed file stay a constant offset of the edited image's S codes (and are saved back)."""
        d = torch.as_tensor(direction, dtype=torch.float32, device=self.device).reshape(1, N_STYLE_CHANNELS, 512)
        self.styles_direction.copy_(d)
        self.delta = d[:, S_TRAINABLE_SPACE_CHANNELS].clone()
        off = d.clone()
        off[:, S_TRAINABLE_SPACE_CHANNELS] = 0
        self._offset = off if bool(off.ne(0).any()) else None

    def _edited(self, styles):
        """The edited image's S codes before the trainable rows: styles + the constant non-T rows of a
        resumed direction (none for a fresh run)."""
        return styles if self._offset is None else styles + self._offset

    def _clip_inputs(self, img, orig):
        """Per CLIP loss, its (target, source) inputs: the unprocessed 224-px images for the default loss, the raw
        generator images for the StyleGAN-NADA losses (they preprocess themselves, clip_loss_nada.py:109-111).
        Either image may be None (not needed by the caller)."""
        raw = [getattr(cl, "takes_raw_images", False) for cl, _ in self.clip_losses]
        tgt = src = None
        if not all(raw):
            tgt = unprocess(img, self.mean, self.std) if img is not None else None
            with torch.no_grad():
                src = unprocess(orig, self.mean, self.std) if orig is not None else None
        return [(img, orig) if r else (tgt, src) for r in raw]

    def _synth_edited(self, styles, d):
        """The edited image: styles (+ a resumed direction's fixed rows) with ``d`` on the trainable rows -- d is
        [1, 8, 512] (find_direction) or [n, 8, 512] (the latent mapper's per-sample delta)."""
        return self.synth_fn(self.G_edit, self.until_k, self._edited(styles), self.temp_shapes_edit, self.noise_mode,
                             delta=d)

    def _original_branch(self, styles):
        """Everything that depends only on the original image (no gradient): its synthesis, its IR-SE50
        features and its CLIP embeddings."""
        with torch.no_grad():
            orig = self.synth_fn(self.G, self.until_k, styles, self.temp_shapes, self.noise_mode)
            y_feats = self.id_loss.target_feats(orig)
            src_embs = [cl.encode_src(s) for (cl, _), (_, s) in zip(self.clip_losses, self._clip_inputs(None, orig))]
        return y_feats, src_embs

    def _pair_terms(self, styles, d, key=None):
        """Batched-loss form: the original image's synthesis (no gradient) runs on the second stream
        beside the edited one (or was already run by the previous iteration's prefetch, `key` = its
        rows); then each loss network sees [edited; original] as one batch."""
        side = self._side_stream()
        pref, self._pref = self._pref, None
        y_feats = src_embs = None
        if side is not None and pref is not None and pref[0] == key:
            main = torch.cuda.current_stream()
            img = self._synth_edited(styles, d)
            main.wait_stream(self._pre)
            orig = pref[1]
            orig.record_stream(main)
            y_feats, src_embs = pref[2], pref[3]
            for t in [y_feats] + (src_embs or []):
                if t is not None:
                    t.record_stream(main)
        elif side is not None:
            main = torch.cuda.current_stream()
            side.wait_stream(main)
            with torch.cuda.stream(side), torch.no_grad():
                orig = self.synth_fn(self.G, self.until_k, styles, self.temp_shapes, self.noise_mode)
            img = self._synth_edited(styles, d)
            main.wait_stream(side)
            orig.record_stream(main)
        else:
            img = self._synth_edited(styles, d)
            with torch.no_grad():
                orig = self.synth_fn(self.G, self.until_k, styles, self.temp_shapes, self.noise_mode)
        if side is not None and getattr(self, "diag_losses_on_main", False):   # diagnostic (tools/det_check.py)
            self._fwd_done = torch.cuda.Event()
            self._fwd_done.record(main)
            id_terms = (self.id_loss.per_sample_with(img, y_feats) if y_feats is not None
                        else self.id_loss.per_sample_pair(img, orig))
            side = None
        elif side is not None:
            # the next iteration's original-image synthesis (prefetch stream) may start from here: it then
            # overlaps the latency-bound loss networks and this iteration's backward
            self._fwd_done = torch.cuda.Event()
            self._fwd_done.record(main)
            # the two loss networks are independent and neither fills the GPU (small GEMMs): IR-SE50 runs on
            # the second stream beside CLIP; autograd runs each backward on its forward's stream and joins
            # them where the gradients meet (d img)
            side.wait_stream(main)
            # every tensor the side stream reads but another stream allocated is recorded on the side stream: freed
            # on the host while the side stream's kernels still read it (y_feats is freed as soon as the backward has
            # used it, and its backward runs on the side stream), its block would otherwise go to the next
            # allocation of its own stream -- the prefetch stream writing the next iteration's image into the
            # features the ID-loss backward is about to read (a hazard found while chasing the pipelined step's
            # run-to-run differences; not their cause)
            img.record_stream(side)
            for t in (y_feats, orig):
                if t is not None:
                    t.record_stream(side)
            with torch.cuda.stream(side):
                id_terms = (self.id_loss.per_sample_with(img, y_feats) if y_feats is not None
                            else self.id_loss.per_sample_pair(img, orig))
        else:
            id_terms = self.id_loss.per_sample_pair(img, orig)
        if src_embs is not None:
            clip_terms = sum(w * cl.per_sample_with(e, t) for (cl, w), (t, _), e in
                             zip(self.clip_losses, self._clip_inputs(img, None), src_embs))
        else:
            clip_terms = sum(w * cl.per_sample_pair(t, s) for (cl, w), (t, s) in zip(self.clip_losses,
                                                                                      self._clip_inputs(img, orig)))
        if side is not None:
            main.wait_stream(side)
            id_terms.record_stream(main)
        return id_terms, clip_terms

    def _local_terms(self, styles, denom, key=None, d=None):
        """Sum-form loss of this rank's shard: every per-sample term / global batch size.  With ``d`` given (the
        latent mapper's per-sample delta): the gradient w.r.t. ``d`` and the 4 summed loss terms.  Without: the
        shard's per-image rows [n, 8*512 + 4] -- image i's gradient w.r.t. the shared direction (the direction
        enters as a per-image leaf, so autograd does not sum over the batch) and its 4 loss terms.

        On the GPU the original-image branch runs on a second HIP stream, concurrently with the edited
        image's synthesis (it shares no data with it), and joins before the losses.
        """
        per_image = d is None
        if per_image:
            d = self.delta.detach().expand(styles.shape[0], -1, -1).clone().requires_grad_(True)
        if self.batch_losses:
            id_terms, clip_terms = self._pair_terms(styles, d, key)
            return self._finish(styles, d, id_terms, clip_terms, denom, per_image)
        side = self._side_stream()
        if side is not None:
            main = torch.cuda.current_stream()
            side.wait_stream(main)
            with torch.cuda.stream(side):
                y_feats, src_embs = self._original_branch(styles)
            img = self._synth_edited(styles, d)
            main.wait_stream(side)
            for t in [y_feats] + src_embs:
                if t is not None:   # NadaTerms.encode_src: None when no term needs the source image
                    t.record_stream(main)
        else:
            img = self._synth_edited(styles, d)
            y_feats, src_embs = self._original_branch(styles)
        id_terms = self.id_loss.per_sample_with(img, y_feats)
        clip_terms = sum(w * cl.per_sample_with(e, t) for (cl, w), e, (t, _) in
                         zip(self.clip_losses, src_embs, self._clip_inputs(img, None)))
        return self._finish(styles, d, id_terms, clip_terms, denom, per_image)

    def _finish(self, styles, d, id_terms, clip_terms, denom, per_image=False):
        T = S_TRAINABLE_SPACE_CHANNELS
        sT = styles.index_select(1, self.t_idx)
        if per_image:
            l2_den = float(denom * len(T) * 512)
            if FUSED_TOTAL:
                total, _ = _LossTotal.apply(id_terms, clip_terms, d, sT, self.coef["id"], self.coef["clip"],
                                            self.coef["l2"], l2_den, float(denom))
            else:
                total = (self.coef["id"] * id_terms.sum() / denom + self.coef["clip"] * clip_terms.sum() / denom +
                         self.coef["l2"] * ((sT + d) - sT).square().sum() / l2_den)
            (g,) = torch.autograd.grad(total, d)
            with torch.no_grad():   # each image's share of the 4 logged terms (sum form)
                diff = ((sT + d) - sT).flatten(1)
                l2 = rowops.row_dot(diff, diff)
                parts = torch.stack([self.coef["clip"] * clip_terms / denom, self.coef["id"] * id_terms / denom,
                                     torch.zeros_like(l2), self.coef["l2"] * l2 / l2_den], 1)
            return torch.cat([g.flatten(1), parts.to(g.dtype)], 1)
        if FUSED_TOTAL:
            total, parts = _LossTotal.apply(id_terms, clip_terms, d, sT, self.coef["id"], self.coef["clip"],
                                            self.coef["l2"], float(denom * len(T) * 512), float(denom))
            (g,) = torch.autograd.grad(total, d)
            return g, parts
        l2_sum = ((sT + d) - sT).square().sum()
        id_part = self.coef["id"] * id_terms.sum() / denom
        clip_part = self.coef["clip"] * clip_terms.sum() / denom
        l2_part = self.coef["l2"] * l2_sum / (denom * len(T) * 512)
        (g,) = torch.autograd.grad(id_part + clip_part + l2_part, d)
        return g, torch.stack([clip_part.detach(), id_part.detach(), torch.zeros_like(l2_part), l2_part.detach()])

    def _side_stream(self):
        if not (self.overlap and self.device.type == "cuda"):
            return None
        if getattr(self, "_side", None) is None:
            self._side = self.stream_factory(self.device)
        return self._side

    def _shard(self, i):
        lo, hi = i * self.B, min((i + 1) * self.B, self.n_items)
        return lo, hi, _dist.shard_rows(lo, hi, self.world.rank, self.world.world_size)

    def _plan(self, n_local):
        """The kernel-plan scope of a shard of n_local images (see plan_batch)."""
        if self.device.type != "cuda":
            return contextlib.nullcontext()
        return _hip.plan_batch(self.plan_batch, n_local)

    def _prefetch_next(self):
        """Draw the next iteration's batch (the same single randint per iteration, one step early) and start
        its original-image synthesis on the third stream once this iteration's forward is done."""
        self._next_i = self.rng.randint(0, self.num_batches)
        _, _, (a, b) = self._shard(self._next_i)
        if b <= a:
            return
        if getattr(self, "_pre", None) is None:
            self._pre = self.stream_factory(self.device)
        self._pre.wait_event(self._fwd_done)
        if getattr(self, "diag_id_after_bwd", False):
            self._diag_id_after = torch.cuda.Event()
            self._diag_id_after.record(torch.cuda.current_stream())
        with torch.cuda.stream(self._pre), torch.no_grad(), self._plan(b - a):
            out = self._prefetch_body(self.styles_array[a:b])
        self._pref = ((a, b),) + out

    def _prefetch_body(self, styles):
        orig = self.synth_fn(self.G, self.until_k, styles, self.temp_shapes, self.noise_mode)
        if self.prefetch_id and getattr(self, "_diag_id_after", None) is not None:
            torch.cuda.current_stream().wait_event(self._diag_id_after)   # diagnostic (tools/det_check.py)
        feats = self.id_loss.target_feats(orig) if self.prefetch_id else None
        embs = None
        if self.prefetch_clip:
            embs = [cl.encode_src(s) for (cl, _), (_, s) in zip(self.clip_losses, self._clip_inputs(None, orig))]
        return orig, feats, embs

    def step(self):
        """One iteration: this rank's per-image rows (local_step), the exchange + fixed-order sum (combine), the
        SGD update (apply_step)."""
        return self.apply_step(self.combine(self.local_step()))

    def local_step(self):
        """This rank's part of an iteration: the batch pick, one [8*512 + 4] row per image of its shard (the
        image's sum-form direction gradient and loss terms; [0, 8*512 + 4] for an empty shard), the next batch's
        prefetch."""
        self.it += 1
        if self._next_i is not None:
            i, self._next_i = self._next_i, None
        else:
            i = self.rng.randint(0, self.num_batches)
        self._cur_i = i
        lo, hi, (a, b) = self._shard(i)
        self._cur_span = (lo, hi)
        self.styles_direction.index_copy_(1, self.t_idx, self.delta)
        pipelined = self.prefetch_orig and self.batch_losses and self._side_stream() is not None
        if b > a:
            with self._plan(b - a):
                rows = self._local_terms(self.styles_array[a:b], hi - lo, key=(a, b))
            if pipelined:
                self._prefetch_next()
        else:
            rows = torch.zeros(0, self.delta.numel() + 4, device=self.device)
            if pipelined:
                self._pref = None
        return rows

    def combine(self, rows):
        """The iteration's [8*512 + 4] buffer from every rank's per-image rows: gathered in global image order
        (World.gather_rows; one rank: the rows themselves) and summed over the global batch in one fixed order --
        the same tensor and the same reduction whatever the number of ranks."""
        lo, hi = self._cur_span
        return self.world.gather_rows(rows, lo, hi).sum(0)

    def apply_step(self, buf):
        """The SGD update from the combined buffer (every rank holds the same one after gather_rows + combine)."""
        lr_t = cosine_lr(self.lr0, self.it, self.total_iterations)
        grad = buf[:-4].view_as(self.delta)
        self.delta = torch.add(self.delta, grad, alpha=-lr_t)  # == torch.optim.SGD step (find_direction.py:339)
        self.last = {"it": self.it, "batch": self._cur_i, "lr": lr_t, "grad": grad, "parts": buf[-4:]}
        return self.last

    def log_line(self):
        p = self.last["parts"].tolist()
        g = self.last["grad"].norm().item()
        return (f"Iteration {self.it}, gradient norm: {g:.4f}, lr {self.last['lr']:.4f}\n"
                f"Total loss: {sum(p):.4f}, clip loss: {p[0]:.4f}, identity loss: {p[1]:.4f}, "
                f"landmarks loss: {p[2]:.4f}, l2 loss: {p[3]:.4f}")

    def save(self, path):
        np.savez(path, s=self.styles_direction.detach().cpu().numpy())


# ------------------------------------------------------------------------------------------- CLI helpers


def load_generator(network, resolution, device, conv_clamp=256):
    """'synthetic' -> seeded config-f / paper256 generator of ``resolution`` px; *.pkl -> the pickle's G_ema
    through the exec-free unpickler (stylemc_amd.legacy, config from its init_kwargs); *.pt/*.pth/
    *.safetensors -> a G_ema state_dict (legacy.py:172-203 names) with the config inferred from its shapes
    (``conv_clamp`` is not stored there).  For a real network ``resolution`` is NOT the generator's size: as
    in the reference it only selects how many blocks are rendered (until_k, find_direction.py:263)."""
    from . import legacy, networks, synthetic
    if network in (None, "", "synthetic"):
        cfg = synthetic.generator_config(resolution=resolution)
        return networks.build_generator(cfg, synthetic.generator_state_dict(cfg, seed=0), device=device)
    if network.startswith("http"):
        raise SystemExit(f"{network}: no network access; download the pickle and pass its local path")
    if not os.path.exists(network):
        raise SystemExit(f"{network}: no such file")
    if network.endswith(".pkl"):
        return legacy.load_generator_pkl(network, device=device)
    if network.endswith(".safetensors"):
        from safetensors.torch import load_file
        sd = load_file(network)
    else:
        sd = torch.load(network, map_location="cpu", weights_only=True)
    sd = {k[len("G_ema."):] if k.startswith("G_ema.") else k: v for k, v in sd.items()}
    return networks.build_generator(networks.infer_generator_config(sd, conv_clamp), sd, device=device)


def until_k_for(G, resolution):
    """Last block index rendered for --resolution (find_direction.py:263 resolution_dict {256: 6, 512: 7,
    1024: 8}, i.e. log2(resolution) - 2), bounded by the generator's own depth."""
    k = RESOLUTION_DICT.get(resolution, int(math.log2(resolution)) - 2)
    last = len(G.synthesis.block_resolutions) - 1
    if k > last:
        raise SystemExit(f"--resolution {resolution} is above the generator's {G.img_resolution} px")
    return k


def load_styles(s_input, n_seeds, device, seed=0):
    from . import synthetic
    if s_input:
        return torch.tensor(np.load(s_input)["s"], device=device, dtype=torch.float32)
    return synthetic.synthetic_styles(n_seeds, seed=seed).to(device)


def _load_weights(path):
    """A state_dict file without code execution: safetensors, or torch.load(weights_only=True)."""
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        return load_file(path)
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(sd, dict) and "state_dict" in sd and isinstance(sd["state_dict"], dict):
        sd = sd["state_dict"]
    return sd


def load_text_features(path):
    """--text_features npz: key 'small' / 'large' per CLIP model, or 'text_features' for both (each
    [1, 512] = norm(E_T(pos) - E_T(neg)) of that model, clip_loss.py:15-18)."""
    with np.load(path) as z:
        if "text_features" in z:
            return {"small": z["text_features"], "large": z["text_features"]}
        return {k: z[k] for k in ("small", "large") if k in z}


def build_clip_losses(clip_type, device, text_prompt, negative_text_prompt, clip_loss_type="default", impl="hip",
                      clip_weights=None, text_features=None, bpe_path=None, synthetic_weights=False):
    """init_clip_loss (find_direction.py:100-122): [(loss, weight)], 'double' -> ViT-B/32 at 1 + ViT-B/16 at 0.5
    (:155,163-166).  clip_loss_type 'default' -> clip_loss.CLIPLoss; 'nada' -> clip_loss_nada.CLIPLoss with the
    directional term, 'nada_global' -> with the global term only (:100-114), each bound to (negative prompt,
    prompt) as (source, target) class (:150-157).  clip_weights / text_features: {'small'|'large': ...}."""
    from .clip_loss import MODEL_NAMES, CLIPLoss
    if clip_loss_type not in ("default", "nada", "nada_global"):
        raise ValueError(f"--clip_loss_type must be default, nada or nada_global, got {clip_loss_type!r}")
    if clip_loss_type != "default" and any(v is not None for v in (text_features or {}).values()):
        raise ValueError("--text_features holds the default loss' prompt direction; the NADA losses encode the "
                         "templated prompts themselves (CLIP weights with the text tower + --clip_bpe)")
    kinds = [("small", 1.0), ("large", 0.5)] if clip_type == "double" else [(clip_type, 1.0)]
    clip_weights = {k: v for k, v in (clip_weights or {}).items() if v}
    text_features = {k: v for k, v in (text_features or {}).items() if v is not None}
    if synthetic_weights and (clip_weights or text_features):
        # real weights for one model and seeded ones for another would give a meaningless mixed direction
        missing = [MODEL_NAMES[k] for k, _ in kinds if k not in clip_weights]
        if missing:
            raise ValueError(f"--clip_type {clip_type}: CLIP weights were given, but not for {', '.join(missing)} "
                             f"(--clip_weights for ViT-B/32, --clip_weights_large for ViT-B/16)")
        synthetic_weights = False
    out = []
    if clip_loss_type != "default":
        from . import clip_loss_nada
        lam = dict(lambda_direction=0.0, lambda_global=1.0) if clip_loss_type == "nada_global" else {}
        for kind, w in kinds:
            path = clip_weights.get(kind)
            loss = clip_loss_nada.CLIPLoss(device, clip_model=MODEL_NAMES[kind], impl=impl, bpe_path=bpe_path,
                                           clip_state_dict=_load_weights(path) if path else None,
                                           synthetic_weights=synthetic_weights, **lam)
            out.append((clip_loss_nada.NadaTerms(loss, negative_text_prompt, text_prompt), w))
        return out
    for kind, w in kinds:
        path = clip_weights.get(kind)
        out.append((CLIPLoss(device, text_prompt, negative_text_prompt, kind, impl=impl,
                             clip_state_dict=_load_weights(path) if path else None,
                             text_features=text_features.get(kind), bpe_path=bpe_path,
                             synthetic_weights=synthetic_weights), w))
    return out


def _cli():
    import click

    @click.command()
    @click.pass_context
    @click.option("--network", "network_pkl", default="synthetic", help="generator state_dict (.pt/.safetensors) or 'synthetic'")
    @click.option("--noise-mode", type=click.Choice(["const", "random", "none"]), default="const", show_default=True)
    @click.option("--s_input", type=str, default=None, metavar="FILE", help="npz with key 's' [n,26,512]")
    @click.option("--outdir", type=str, required=True, default="runs/male2female_id0.75_clip1.0_lr2.5_power2.0/")
    @click.option("--text_prompt", type=str, required=True, default="a photo of a face of a feminine woman with no makeup")
    @click.option("--negative_text_prompt", type=str, default="a photo of a face of a masculine man")
    @click.option("--clip_type", type=str, default="double")
    @click.option("--clip_loss_type", type=str, default="default")
    @click.option("--resolution", type=int, default=256)
    @click.option("--batch_size", type=int, default=4)
    @click.option("--learning_rate", type=float, default=1.5)
    @click.option("--n_epochs", type=int, default=4)
    @click.option("--resume", type=str, default=None)
    @click.option("--identity_loss_coef", type=float, default=0.6)
    @click.option("--landmarks_loss_coef", type=float, default=25.0)
    @click.option("--l2_reg_coef", type=float, default=0.1)
    @click.option("--clip_loss_coef", type=float, default=1.0)
    @click.option("--n_seeds", type=int, default=129, help="rows of synthetic S when --s_input is absent")
    @click.option("--seed", type=int, default=0, help="seed of the batch picker (unseeded in the reference)")
    @click.option("--per_gpu_batch", is_flag=True, help="throughput mode: global batch = batch_size x world")
    @click.option("--max_iterations", type=int, default=None)
    @click.option("--init_std", type=float, default=0.01, help="std of the seeded start direction (0 = reference)")
    @click.option("--clip_weights", type=str, default=None, help="OpenAI CLIP ViT-B/32 state_dict (.pt/.safetensors)")
    @click.option("--clip_weights_large", type=str, default=None, help="OpenAI CLIP ViT-B/16 state_dict (clip_type large/double)")
    @click.option("--clip_bpe", type=str, default=None, help="CLIP BPE merges file (bpe_simple_vocab_16e6.txt.gz)")
    @click.option("--text_features", type=str, default=None, help="npz of precomputed text directions ('small'/'large')")
    @click.option("--id_weights", type=str, default="id_loss/model_ir_se50.pth", show_default=True)
    @click.option("--conv_clamp", type=float, default=256.0, help="conv_clamp of a state_dict network (not stored in it)")
    @click.option("--allow_synthetic_losses", is_flag=True,
                  help="seeded synthetic CLIP / IR-SE50 weights (implied by --network synthetic)")
    @click.option("--impl", type=click.Choice(["hip", "torch"]), default="hip",
                  help="loss networks on the gfx950 kernels (hip) or PyTorch-ROCm ops (torch)")
    def find_direction(ctx, network_pkl, noise_mode, s_input, outdir, text_prompt, negative_text_prompt, clip_type,
                       clip_loss_type, resolution, batch_size, learning_rate, n_epochs, resume, identity_loss_coef,
                       landmarks_loss_coef, l2_reg_coef, clip_loss_coef, n_seeds, seed, per_gpu_batch, max_iterations,
                       init_std, clip_weights, clip_weights_large, clip_bpe, text_features, id_weights, conv_clamp,
                       allow_synthetic_losses, impl):
        from .id_loss import IDLoss
        world = _dist.init_from_env(use_cuda=True)
        device = torch.device("cuda", world.device_index)
        torch.cuda.set_device(device)
        if landmarks_loss_coef != 0:
            warnings.warn("landmarks loss adds no gradient in the reference (no_grad, find_direction.py:90); ignored")
        synthetic_losses = allow_synthetic_losses or network_pkl in (None, "", "synthetic")
        G = load_generator(network_pkl, resolution, device, conv_clamp=conv_clamp)
        until_k_for(G, resolution)
        os.makedirs(outdir, exist_ok=True)
        styles_array = load_styles(s_input, n_seeds, device)
        clips = build_clip_losses(clip_type, device, text_prompt, negative_text_prompt, clip_loss_type, impl=impl,
                                  clip_weights={"small": clip_weights, "large": clip_weights_large},
                                  text_features=load_text_features(text_features) if text_features else None,
                                  bpe_path=clip_bpe, synthetic_weights=synthetic_losses)
        if synthetic_losses and not os.path.exists(id_weights or ""):
            id_weights = None
            if world.rank == 0:
                warnings.warn("IR-SE50 / CLIP: seeded synthetic weights where none were given (synthetic run)")
        finder = DirectionFinder(
            G, styles_array, clips,
            IDLoss("a", device=device, weights=id_weights, impl=impl), resolution=resolution, batch_size=batch_size,
            learning_rate=learning_rate,
            n_epochs=n_epochs, identity_loss_coef=identity_loss_coef, l2_reg_coef=l2_reg_coef,
            clip_loss_coef=clip_loss_coef, noise_mode=noise_mode, seed=seed, world=world,
            global_batch=batch_size * world.world_size if per_gpu_batch else batch_size,
            init_delta=initial_delta(seed, init_std) if init_std > 0 else None)
        if resume:
            finder.load_direction(np.load(resume)["s"])
        if world.rank == 0:
            print(f"training param shape {tuple(finder.delta.shape)}")
            print(f"Total number of iterations: {finder.total_iterations}")
        t1 = time.time()
        total = finder.total_iterations if max_iterations is None else min(max_iterations, finder.total_iterations)
        for _ in range(total):
            finder.step()
            if world.rank == 0 and finder.it % 1000 == 999:
                finder.save(f"{outdir}/direction_last.npz")
            if world.rank == 0 and finder.it % 10 == 0:
                print(finder.log_line())
        if world.rank == 0:
            finder.save(f'{outdir}/direction_{text_prompt.replace(" ", "_")}.npz')
            print("time passed:", time.time() - t1)

    return find_direction


def main():
    _cli()()


if __name__ == "__main__":
    main()
