"""CPU restatement of generate_fromS.py:89-207 (no blending) -- TEST ORACLE ONLY.

For each item i and power p in [0, change_power]: styles += dir*p (all rows, in place, :166),
render styles[[i]] (:172-173), uint8((img*127.5 + 128).clamp(0, 255)) (:174-175), styles -= dir*p (:204).
With a mapper the direction is rebuilt per (item, power) from mapper(styles[i, T]) (:149-165, whitelist
threshold 0.1 and the STOPLIST ids :153-162).  --projected-w: G.synthesis(w) per W row (:89-102).
"""
import torch

from .synthesis import generate_image


def to_uint8(img):
    return (img.permute(0, 2, 3, 1) * 127.5 + 128).clamp(0, 255).to(torch.uint8)


STOPLIST_S_IDS = [4863, 6247, 4943, 4724, 3114, 4623, 4726]
T = [2, 3, 5, 6, 8, 9, 11, 12]


def mapper_direction(mapper, styles_i, use_whitelist):
    styles_direction = torch.zeros(1, 26, 512)
    delta = mapper(styles_i[T].unsqueeze(0))
    if use_whitelist:
        delta[delta.abs() < 0.1] = 0.0
    styles_direction[:, T] = delta
    if use_whitelist:
        mask = torch.zeros(26 * 512, dtype=torch.bool)
        mask[STOPLIST_S_IDS] = True
        styles_direction[mask.view(*styles_direction.size())] = 0.0
    return styles_direction


@torch.no_grad()
def render_projected_w(G, ws, noise_mode="const"):
    return [to_uint8(G.synthesis(w.unsqueeze(0), noise_mode=noise_mode))[0] for w in ws]


@torch.no_grad()
def render_pairs(G, styles, direction, change_power, temp_shapes, noise_mode="const", mapper=None,
                 use_whitelist=False, G2=None, temp_shapes2=None):
    """G2: --network2, the edited image (j == 1) from the second generator (:80-86,168-170)."""
    out = []
    for i in range(styles.shape[0]):
        imgs = []
        for j, p in enumerate([0, change_power]):
            if mapper is not None:
                direction = mapper_direction(mapper, styles[i], use_whitelist)
            styles += direction * p
            if G2 is not None and j == 1:
                _, img = generate_image(G2, 100, styles[[i]], temp_shapes2, noise_mode)
            else:
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
