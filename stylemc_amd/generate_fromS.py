"""generate_fromS on MI355X: drop-in for the reference's generate_fromS.py.

Restates generate_fromS.py:58-209:
  * --projected-w FILE (:89-102): every W row through G.synthesis -> proj{idx:02d}.png, then return
  * styles = np.load(s_input)['s'][:n]; the direction is either the global
    ``{outdir}/direction_{prompt}.npz`` (:123-126) or, with --use_mapper 1, per item
    ``mapper(styles[i, T])`` from ``{outdir}/mapper_{prompt}.pth`` (:117-122,149-165; Mapper(neg_slope =
    --mapper_neg_slope)), with --use_whitelist: |delta| < 0.1 -> 0 and the STOPLIST S ids zeroed (:153-162)
  * for each item i, for p in [0, change_power]:  styles += direction * p   (ALL rows, in place, :166)
        img = generate_image(G, 100, styles[[i]]);  uint8((img*127.5 + 128).clamp(0, 255))  (:172-175)
        styles -= direction * p                                                            (:204)
    -- the in-place add/subtract pair is replayed exactly, so its fp32 drift over the items matches
  * JPEG (quality 95) of [original | edited] per item (:206-207)
New (README.md:54-56 names a video flag the reference never implemented): ``--from_video N`` renders
N frames per item with power linspace(0, change_power, N) (no in-place drift: styles[i] + d*p), batched
on the GPU, written as JPEG frames + one uint8 .npy stack per item.
--network2 (:42-43,80-86,168-170): the edited image (j = 1, power change_power) is rendered by a second generator
G2 with its own temp shapes; the original (power 0) by G.  In the video sweep, power-0 frames come from G and
every other frame from G2.
Out of scope: deeplab feature blending (--use_blending).
"""
import os
import time

import numpy as np
import torch

from . import utils


def to_uint8(img):
    """generate_fromS.py:174-175: (img*127.5 + 128).clamp(0,255) -> uint8 (truncation), NHWC."""
    return (img.permute(0, 2, 3, 1) * 127.5 + 128).clamp(0, 255).to(torch.uint8)


STOPLIST_S_IDS = [4863, 6247, 4943, 4724, 3114, 4623, 4726]        # generate_fromS.py:36


def mapper_direction(mapper, style_row, use_whitelist=False):
    """generate_fromS.py:149-162: [1, 26, 512] direction from the mapper's delta on the T rows."""
    T = utils.S_TRAINABLE_SPACE_CHANNELS
    d = torch.zeros(1, utils.N_STYLE_CHANNELS, 512, device=style_row.device)
    delta = mapper(style_row[T].unsqueeze(0))
    if use_whitelist:
        delta = delta.masked_fill(delta.abs() < 0.1, 0.0)
    d[:, T] = delta
    if use_whitelist:
        d.view(-1)[torch.as_tensor(STOPLIST_S_IDS, device=d.device)] = 0.0
    return d


@torch.no_grad()
def render_projected_w(G, ws, noise_mode="const"):
    """generate_fromS.py:89-102: yield (idx, uint8 HWC) of G.synthesis(w) per W row."""
    for idx, w in enumerate(ws):
        yield idx, to_uint8(G.synthesis(w.unsqueeze(0), noise_mode=noise_mode))[0]


@torch.no_grad()
def render_pairs(G, styles, direction, change_power, temp_shapes, noise_mode="const", until_k=100, mapper=None,
                 use_whitelist=False, G2=None, temp_shapes2=None):
    """Yield (i, [orig_uint8, edited_uint8]) replaying the reference's in-place styles drift.  direction is
    the global [1, 26, 512] direction, or None with a ``mapper`` (per-item direction).  G2 (--network2): the
    generator of the edited image (generate_fromS.py:168-170)."""
    for i in range(styles.shape[0]):
        imgs = []
        for j, p in enumerate([0, change_power]):
            if mapper is not None:
                direction = mapper_direction(mapper, styles[i], use_whitelist)
            styles += direction * p
            g, ts = (G2, temp_shapes2) if (G2 is not None and j == 1) else (G, temp_shapes)
            _, img = utils.generate_image(g, until_k, styles[[i]], ts, noise_mode)
            imgs.append(to_uint8(img)[0])
            styles -= direction * p
        yield i, imgs


@torch.no_grad()
def render_sweep(G, style_row, direction, powers, temp_shapes, noise_mode="const", batch=8, until_k=100, G2=None,
                 temp_shapes2=None):
    """Frames for one S row along the direction: uint8 [len(powers), H, W, 3].  G2: renders every frame whose
    power is not 0 (the edited frames; --network2)."""
    powers = [float(p) for p in np.asarray(powers, dtype=np.float64)]
    groups = [(G, temp_shapes, [k for k, p in enumerate(powers) if G2 is None or p == 0.0])]
    if G2 is not None:
        groups.append((G2, temp_shapes2, [k for k, p in enumerate(powers) if p != 0.0]))
    out = [None] * len(powers)
    pw = torch.as_tensor(powers, dtype=torch.float32, device=style_row.device)
    for g, ts, ks in groups:
        for lo in range(0, len(ks), batch):
            idx = ks[lo:lo + batch]
            p = pw[torch.as_tensor(idx, device=style_row.device)].view(-1, 1, 1)
            s = style_row.unsqueeze(0) + direction * p
            _, img = utils.generate_image(g, until_k, s, ts, noise_mode)
            for k, fr in zip(idx, to_uint8(img)):
                out[k] = fr
    return torch.stack(out)


def _cli():
    import click

    @click.command()
    @click.option("--network", "network_pkl", default="synthetic",
                  help="network pickle / G_ema state_dict, or 'synthetic'")
    @click.option("--network2", "network2_pkl", default=None,
                  help="second generator for the edited image (default: --network)")
    @click.option("--noise-mode", type=click.Choice(["const", "random", "none"]), default="const", show_default=True)
    @click.option("--projected-w", "projected_w", type=str, default=None, metavar="FILE",
                  help="npz with key 'w' [n, num_ws, 512]: render each W with G.synthesis")
    @click.option("--s_input", type=str, default=None, metavar="FILE")
    @click.option("--use_mapper", type=int, default=0)
    @click.option("--n", type=int, default=99999)
    @click.option("--outdir", type=str, required=True)
    @click.option("--text_prompt", type=str, required=True)
    @click.option("--change_power", type=float, default=2.0)
    @click.option("--mapper_neg_slope", type=float, default=0.01, help="mapper hyperparam (leaky relu slope)")
    @click.option("--use_blending", type=int, default=0)
    @click.option("--use_whitelist", type=int, default=0)
    @click.option("--resolution", type=int, default=1024, help="resolution of the synthetic generator")
    @click.option("--conv_clamp", type=float, default=256.0, help="conv_clamp of a state_dict network")
    @click.option("--from_video", type=int, default=0, help="frames per item for a 0 -> change_power sweep")
    @click.option("--video_batch", type=int, default=8)
    def generate_images(network_pkl, network2_pkl, noise_mode, projected_w, s_input, use_mapper, n, outdir,
                        text_prompt, change_power, mapper_neg_slope, use_blending, use_whitelist, resolution, conv_clamp,
                        from_video, video_batch):
        from PIL import Image

        from .find_direction import load_generator
        if use_blending:
            raise SystemExit("deeplab feature blending (--use_blending) is outside the hot path")
        device = torch.device("cuda")
        G = load_generator(network_pkl, resolution, device, conv_clamp=conv_clamp)
        G2 = temp_shapes2 = None
        if network2_pkl and network2_pkl != network_pkl:
            print("using 2 generators")
            G2 = load_generator(network2_pkl, resolution, device, conv_clamp=conv_clamp)
            temp_shapes2 = utils.get_temp_shapes(G2)
        os.makedirs(outdir, exist_ok=True)
        stem = text_prompt.replace(" ", "_")
        if projected_w is not None:
            ws = torch.tensor(np.load(projected_w)["w"][:n], device=device)
            if tuple(ws.shape[1:]) != (G.num_ws, G.w_dim):
                raise SystemExit(f"{projected_w}: w {tuple(ws.shape)} does not match G ({G.num_ws}, {G.w_dim})")
            for idx, img in render_projected_w(G, ws, noise_mode):
                Image.fromarray(img.cpu().numpy(), "RGB").save(f"{outdir}/proj{idx:02d}.png")
            return
        if s_input is None:
            raise SystemExit("--s_input (or --projected-w) is required")
        temp_shapes = utils.get_temp_shapes(G)
        styles = torch.tensor(np.load(s_input)["s"][:n], device=device)
        mapper = direction = None
        if use_mapper:
            from .latent_mappers import Mapper
            mapper = Mapper(neg_slope=mapper_neg_slope).eval()
            mapper.load_state_dict(torch.load(f"{outdir}/mapper_{stem}.pth", map_location="cpu", weights_only=True))
            mapper = mapper.to(device)
        else:
            direction = torch.tensor(np.load(f"{outdir}/direction_{stem}.npz")["s"], device=device)
        t1 = time.time()
        if from_video:
            powers = np.linspace(0.0, change_power, from_video)
            for i in range(styles.shape[0]):
                d = mapper_direction(mapper, styles[i], use_whitelist) if mapper is not None else direction
                frames = render_sweep(G, styles[i], d, powers, temp_shapes, noise_mode, video_batch, G2=G2,
                                      temp_shapes2=temp_shapes2)
                arr = frames.cpu().numpy()
                base = f"{outdir}/{stem}_{i:03d}"
                np.save(base + "_frames.npy", arr)
                for k, fr in enumerate(arr):
                    Image.fromarray(fr, "RGB").save(f"{base}_f{k:03d}.jpeg", quality=95)
        else:
            for i, imgs in render_pairs(G, styles, direction, change_power, temp_shapes, noise_mode, mapper=mapper,
                                        use_whitelist=bool(use_whitelist), G2=G2, temp_shapes2=temp_shapes2):
                arr = np.concatenate([im.cpu().numpy() for im in imgs], axis=1)
                Image.fromarray(arr, "RGB").save(f"{outdir}/{stem}_{i:03d}.jpeg", quality=95)
        print("time passed:", time.time() - t1)

    return generate_images


def main():
    _cli()()


if __name__ == "__main__":
    main()
