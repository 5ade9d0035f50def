"""Seeds -> W -> S: producers of ``--s_input`` for find_direction.

  seeds_to_w  <- generate_w.py:46-51   z_s = RandomState(seed).randn(1, z_dim) (float64, as drawn there),
                                       ws = G.mapping(z, c, truncation_psi)  -> npz key 'w' [n, num_ws, 512]
  w_to_s      <- w_s_converter.py:75-82 + utils.py:77-87,123-158: split_ws, every layer's affine FC,
                                       packed [n, 26, 512] zero padded -> npz key 's' (mutates G: affines
                                       become Identity, like the reference)
The mapping's lrelu FCs run through the HIP bias_act kernel; the affines are plain addmm.

    python -m stylemc_amd.w_s generate_w --seeds 1-129 --trunc 0.7 --out_file projected_w.npz
    python -m stylemc_amd.w_s w_s_converter --projected-w projected_w.npz --out_file s.npz
"""
import os

import numpy as np
import torch

from . import utils
from .synthetic import seed_latents


def parse_seeds(text):
    """--seeds as generate_w.py takes them (utils.py:64-74 num_range): comma-separated items, each a seed or an
    inclusive range 'a-b'."""
    out = []
    for item in str(text).split(","):
        lo, sep, hi = item.strip().partition("-")
        out.extend(range(int(lo), int(hi) + 1) if sep else [int(lo)])
    return out


@torch.no_grad()
def seeds_to_w(G, seeds, truncation_psi=1.0, device="cuda"):
    z = seed_latents(seeds, G.z_dim).to(device)
    return G.mapping(z, None, truncation_psi=truncation_psi)


@torch.no_grad()
def w_to_s(G, ws):
    styles, _ = utils.get_styles(G, ws, utils.split_ws(G, ws))
    return styles


def _cli():
    import click

    from .find_direction import load_generator

    @click.group()
    def cli():
        pass

    @cli.command("generate_w")
    @click.option("--network", "network_pkl", default="synthetic")
    @click.option("--seeds", type=parse_seeds, required=True)
    @click.option("--trunc", "truncation_psi", type=float, default=1.0, show_default=True)
    @click.option("--out_file", type=str, default="encoder4editing/projected_w.npz")
    @click.option("--resolution", type=int, default=1024)
    def generate_w(network_pkl, seeds, truncation_psi, out_file, resolution):
        G = load_generator(network_pkl, resolution, "cuda")
        ws = seeds_to_w(G, seeds, truncation_psi)
        os.makedirs(os.path.dirname(out_file) or ".", exist_ok=True)
        np.savez(out_file, w=ws.cpu().numpy())

    @cli.command("w_s_converter")
    @click.option("--network", "network_pkl", default="synthetic")
    @click.option("--projected-w", "projected_w", type=str, required=True)
    @click.option("--out_file", type=str, default="out/input.npz")
    @click.option("--resolution", type=int, default=1024)
    def w_s_converter(network_pkl, projected_w, out_file, resolution):
        G = load_generator(network_pkl, resolution, "cuda")
        ws = torch.tensor(np.load(projected_w)["w"], device="cuda")
        os.makedirs(os.path.dirname(out_file) or ".", exist_ok=True)
        np.savez(out_file, s=w_to_s(G, ws).cpu().numpy())

    return cli


if __name__ == "__main__":
    _cli()()
