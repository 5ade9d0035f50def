"""generate_fromS on MI355X: drop-in for the reference's generate_fromS.py (global-direction path).

Restates generate_fromS.py:58-209 for ``--use_mapper 0 --use_blending 0``:
  * styles = np.load(s_input)['s'][:n]; direction = np.load(f'{outdir}/direction_{prompt}.npz')['s']
  * for each item i, for p in [0, change_power]:  styles += direction * p   (ALL rows, in place, :166)
        img = generate_image(G, 100, styles[[i]]);  uint8((img*127.5 + 128).clamp(0, 255))  (:172-175)
        styles -= direction * p                                                            (:204)
    -- the in-place add/subtract pair is replayed exactly, so its fp32 drift over the items matches
  * JPEG (quality 95) of [original | edited] per item (:206-207)
New (README.md:54-56 names a video flag the reference never implemented): ``--from_video N`` renders
N frames per item with power linspace(0, change_power, N) (no in-place drift: styles[i] + d*p), batched
on the GPU, written as JPEG frames + one uint8 .npy stack per item.
The latent-mapper (--use_mapper) and deeplab blending (--use_blending) paths are out of scope.
"""
import os
import time

import numpy as np
import torch

from . import utils


def to_uint8(img):
    """generate_fromS.py:174-175: (img*127.5 + 128).clamp(0,255) -> uint8 (truncation), NHWC."""
    return (img.permute(0, 2, 3, 1) * 127.5 + 128).clamp(0, 255).to(torch.uint8)


@torch.no_grad()
def render_pairs(G, styles, direction, change_power, temp_shapes, noise_mode="const", until_k=100):
    """Yield (i, [orig_uint8, edited_uint8]) replaying the reference's in-place styles drift."""
    for i in range(styles.shape[0]):
        imgs = []
        for p in [0, change_power]:
            styles += direction * p
            _, img = utils.generate_image(G, until_k, styles[[i]], temp_shapes, noise_mode)
            imgs.append(to_uint8(img)[0])
            styles -= direction * p
        yield i, imgs


@torch.no_grad()
def render_sweep(G, style_row, direction, powers, temp_shapes, noise_mode="const", batch=8, until_k=100):
    """Frames for one S row along the direction: uint8 [len(powers), H, W, 3]."""
    out = []
    powers = torch.as_tensor(powers, dtype=torch.float32, device=style_row.device)
    for lo in range(0, len(powers), batch):
        p = powers[lo:lo + batch].view(-1, 1, 1)
        s = style_row.unsqueeze(0) + direction * p
        _, img = utils.generate_image(G, until_k, s, temp_shapes, noise_mode)
        out.append(to_uint8(img))
    return torch.cat(out)


def _cli():
    import click

    @click.command()
    @click.option("--network", "network_pkl", default="synthetic", help="generator state_dict or 'synthetic'")
    @click.option("--network2", "network2_pkl", default=None, help="(unsupported: second generator)")
    @click.option("--noise-mode", type=click.Choice(["const", "random", "none"]), default="const", show_default=True)
    @click.option("--s_input", type=str, required=True, metavar="FILE")
    @click.option("--use_mapper", type=int, default=0)
    @click.option("--n", type=int, default=99999)
    @click.option("--outdir", type=str, required=True)
    @click.option("--text_prompt", type=str, required=True)
    @click.option("--change_power", type=float, default=2.0)
    @click.option("--use_blending", type=int, default=0)
    @click.option("--use_whitelist", type=int, default=0)
    @click.option("--resolution", type=int, default=1024, help="resolution of the synthetic generator")
    @click.option("--from_video", type=int, default=0, help="frames per item for a 0 -> change_power sweep")
    @click.option("--video_batch", type=int, default=8)
    def generate_images(network_pkl, network2_pkl, noise_mode, s_input, use_mapper, n, outdir, text_prompt,
                        change_power, use_blending, use_whitelist, resolution, from_video, video_batch):
        from PIL import Image

        from .find_direction import load_generator
        if use_mapper or use_blending or use_whitelist or (network2_pkl and network2_pkl != network_pkl):
            raise SystemExit("mapper / blending / whitelist / second-generator paths are outside the hot path")
        device = torch.device("cuda")
        G = load_generator(network_pkl, resolution, device)
        temp_shapes = utils.get_temp_shapes(G)
        styles = torch.tensor(np.load(s_input)["s"][:n], device=device)
        direction = torch.tensor(np.load(f'{outdir}/direction_{text_prompt.replace(" ", "_")}.npz')["s"],
                                 device=device)
        os.makedirs(outdir, exist_ok=True)
        t1 = time.time()
        if from_video:
            powers = np.linspace(0.0, change_power, from_video)
            for i in range(styles.shape[0]):
                frames = render_sweep(G, styles[i], direction, powers, temp_shapes, noise_mode, video_batch)
                arr = frames.cpu().numpy()
                stem = f'{outdir}/{text_prompt.replace(" ", "_")}_{i:03d}'
                np.save(stem + "_frames.npy", arr)
                for k, fr in enumerate(arr):
                    Image.fromarray(fr, "RGB").save(f"{stem}_f{k:03d}.jpeg", quality=95)
        else:
            for i, imgs in render_pairs(G, styles, direction, change_power, temp_shapes, noise_mode):
                arr = np.concatenate([im.cpu().numpy() for im in imgs], axis=1)
                Image.fromarray(arr, "RGB").save(f'{outdir}/{text_prompt.replace(" ", "_")}_{i:03d}.jpeg',
                                                 quality=95)
        print("time passed:", time.time() - t1)

    return generate_images


def main():
    _cli()()


if __name__ == "__main__":
    main()
