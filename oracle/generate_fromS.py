"""CPU restatement of generate_fromS.py:137-207 (global direction, no mapper / blending) -- TEST ORACLE ONLY.

For each item i and power p in [0, change_power]: styles += dir*p (all rows, in place, :166),
render styles[[i]] (:172-173), uint8((img*127.5 + 128).clamp(0, 255)) (:174-175), styles -= dir*p (:204).
"""
import torch

from .synthesis import generate_image


def to_uint8(img):
    return (img.permute(0, 2, 3, 1) * 127.5 + 128).clamp(0, 255).to(torch.uint8)


@torch.no_grad()
def render_pairs(G, styles, direction, change_power, temp_shapes, noise_mode="const"):
    out = []
    for i in range(styles.shape[0]):
        imgs = []
        for p in [0, change_power]:
            styles += direction * p
            _, img = generate_image(G, 100, styles[[i]], temp_shapes, noise_mode)
            imgs.append(to_uint8(img)[0])
            styles -= direction * p
        out.append(imgs)
    return out


@torch.no_grad()
def render_sweep(G, style_row, direction, powers, temp_shapes, noise_mode="const"):
    """Video frames (the README's --from_video, never implemented in the reference): styles[i] + dir*p."""
    powers = torch.as_tensor(powers, dtype=torch.float32).view(-1, 1, 1)
    _, img = generate_image(G, 100, style_row.unsqueeze(0) + direction * powers, temp_shapes, noise_mode)
    return to_uint8(img)
