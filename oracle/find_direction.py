"""CPU restatement of the find_direction optimisation loop (TEST ORACLE ONLY).

Restates find_direction.py:259-351 (the hot loop at :292-347) with the intended behaviour (the
shipped script cannot run: generate_image is called without ``device``, find_direction.py:309):

  * cosine lr:  lr_t = 0.5*lr0*(1 + cos(pi*t/T)),  T = n_epochs*ceil(n/bs)        (:297-301)
  * batch pick: i = np.random.randint(0, ceil(n/bs)) with replacement; seeded here  (:303-304)
  * styles2 = styles + direction, direction rows T = trainable delta                (:307-308)
  * two syntheses (edited, original), compute_loss, backward, SGD p -= lr_t * g      (:309-339)
  * the returned direction is ``styles_direction`` as the reference saves it (:349-351): the delta
    written into it at the start of the LAST iteration (the final SGD step is not copied back).
  * ``init_delta``: the reference starts from exactly zero, where img == original and the directional
    CLIP term normalises a zero vector (clip_loss.py:29-30 -> NaN); runs start from a seeded small
    direction instead (stylemc_amd.find_direction.initial_delta).
"""
import math
import time

import numpy as np
import torch

from .losses import compute_loss, get_mean_std
from .synthesis import N_STYLE_CHANNELS, S_TRAINABLE_SPACE_CHANNELS, generate_image


def cosine_lr(lr0, it, total):
    return float(np.cos(np.pi * it / total) * lr0 * 0.5 + lr0 * 0.5)


def find_direction(G, styles_array, clip_loss, id_loss, temp_shapes, until_k, batch_size=4, learning_rate=1.5,
                   n_epochs=4, identity_loss_coef=0.6, l2_reg_coef=0.1, clip_loss_coef=1.0, noise_mode="const",
                   seed=0, max_iterations=None, log=None, init_delta=None, init_direction=None, clip_loss2=None,
                   clip_loss_type="default", text_prompt=None, negative_text_prompt=None):
    """init_direction: a resumed [1, 26, 512] styles_direction (find_direction.py:266-271); its T rows are the
    start delta and the whole tensor is added to the styles (styles2 = styles + styles_direction, :307-308).
    clip_loss2 / clip_loss_type / prompts: compute_loss's --clip_type double and NADA options (:150-169)."""
    T = S_TRAINABLE_SPACE_CHANNELS
    rng = np.random.RandomState(seed)
    mean, std = get_mean_std()
    n_items = styles_array.shape[0]
    num_batches = math.ceil(n_items / batch_size)
    total = num_batches * n_epochs
    styles_direction = torch.zeros(1, N_STYLE_CHANNELS, 512)
    if init_direction is not None:
        styles_direction = init_direction.detach().clone().reshape(1, N_STYLE_CHANNELS, 512).float()
    delta = styles_direction[:, T].clone()
    if init_delta is not None:  # see stylemc_amd.find_direction.initial_delta: zero start is 0/0 in CLIP
        delta = init_delta.detach().clone().reshape(1, len(T), 512).float()
    delta.requires_grad_(True)
    it = 0
    for _ in range(n_epochs):
        for _ in range(num_batches):
            it += 1
            lr_t = cosine_lr(learning_rate, it, total)
            i = rng.randint(0, num_batches)
            styles = styles_array[i * batch_size:(i + 1) * batch_size]
            with torch.no_grad():
                styles_direction[:, T] = delta
            fixed = styles_direction.clone()
            fixed[:, T] = 0
            styles2 = styles + fixed + _scatter_rows(delta, T)
            _, img = generate_image(G, until_k, styles2, temp_shapes, noise_mode)
            with torch.no_grad():
                _, original_img = generate_image(G, until_k, styles, temp_shapes, noise_mode)
            loss, parts = compute_loss(img, original_img, styles, styles2, clip_loss, id_loss, mean, std,
                                       identity_loss_coef, clip_loss_coef, l2_reg_coef, T, clip_loss2=clip_loss2,
                                       clip_loss_type=clip_loss_type, text_prompt=text_prompt,
                                       negative_text_prompt=negative_text_prompt)
            delta.grad = None
            loss.backward()
            with torch.no_grad():
                delta.add_(delta.grad, alpha=-lr_t)
            if log is not None:
                log.append({"it": it, "batch": i, "lr": lr_t, "loss": float(loss.detach()), "t": time.perf_counter(),
                            "grad_norm": float(delta.grad.norm()), **{k: float(torch.as_tensor(v).detach()) for k, v in parts.items()}})
            if max_iterations is not None and it >= max_iterations:
                return styles_direction, delta.detach()
    return styles_direction, delta.detach()


def _scatter_rows(delta, rows):
    """[1, 8, 512] trainable rows -> [1, 26, 512] direction (differentiable)."""
    full = torch.zeros(1, N_STYLE_CHANNELS, 512, dtype=delta.dtype)
    index = torch.tensor(rows).view(1, -1, 1).expand(1, len(rows), 512)
    return full.scatter(1, index, delta)
