"""generate_fromS (pairs with the reference's in-place drift, and the video sweep) and seeds -> W -> S on
the GPU vs the CPU oracle.  Per-pixel tolerance on the uint8 images (generate_fromS.py:174-175 truncates):
|diff| <= 1 everywhere and >= 99.9 % of pixels exact (fp32 summation order can move a value across an
integer boundary)."""
import numpy as np
import pytest
import torch

from oracle import generate_fromS as OG
from oracle import networks as ON
from oracle import synthesis as OS
from stylemc_amd import synthetic

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _pair(res, cbase):
    from stylemc_amd import build, networks
    build.build(verbose=False)
    cfg = synthetic.generator_config(resolution=res, channel_base=cbase)
    sd = synthetic.generator_state_dict(cfg, seed=0)
    G = networks.build_generator(cfg, sd, device=DEV)
    Go = ON.Generator(512, 0, 512, res, 3, channel_base=cbase, conv_clamp=cfg["conv_clamp"])
    r = Go.load_state_dict(sd, strict=False)
    assert not r.unexpected_keys
    return G, Go.eval().requires_grad_(False)


def _check_u8(a, b, what):
    a = a.cpu().numpy().astype(np.int16)
    b = b.numpy().astype(np.int16)
    diff = np.abs(a - b)
    assert diff.max() <= 1, f"{what}: max |diff| {diff.max()}"
    assert (diff == 0).mean() >= 0.999, f"{what}: exact fraction {(diff == 0).mean():.5f}"


@pytest.mark.parametrize("res,cbase,n", [(32, 512, 4), (1024, 32768, 2)])
def test_generate_fromS_pairs_vs_oracle(res, cbase, n):
    from stylemc_amd import generate_fromS, utils
    G, Go = _pair(res, cbase)
    styles = synthetic.synthetic_styles(n, seed=9)
    direction = torch.zeros(1, 26, 512)
    direction[:, utils.S_TRAINABLE_SPACE_CHANNELS] = torch.randn(1, 8, 512, generator=torch.Generator().manual_seed(1)) * 0.3
    got = list(generate_fromS.render_pairs(G, styles.to(DEV), direction.to(DEV), 2.0, utils.get_temp_shapes(G)))
    ref = OG.render_pairs(Go, styles.clone(), direction, 2.0, OS.get_temp_shapes(Go))
    for (i, imgs), rimgs in zip(got, ref):
        for k in range(2):
            _check_u8(imgs[k], rimgs[k], f"item {i} power {k}")


def test_generate_fromS_video_sweep_vs_oracle():
    from stylemc_amd import generate_fromS, utils
    G, Go = _pair(1024, 32768)
    style_row = synthetic.synthetic_styles(1, seed=3)[0]
    direction = torch.zeros(1, 26, 512)
    direction[:, utils.S_TRAINABLE_SPACE_CHANNELS] = torch.randn(1, 8, 512, generator=torch.Generator().manual_seed(2)) * 0.1
    powers = np.linspace(0.0, 50.0, 5)
    got = generate_fromS.render_sweep(G, style_row.to(DEV), direction.to(DEV), powers, utils.get_temp_shapes(G),
                                      batch=4)
    ref = OG.render_sweep(Go, style_row, direction, powers, OS.get_temp_shapes(Go))
    assert got.shape == (5, 1024, 1024, 3)
    _check_u8(got, ref, "sweep")


def test_seeds_to_w_to_s_vs_oracle():
    from stylemc_amd import w_s
    G, Go = _pair(1024, 32768)
    seeds = [1, 2, 129]
    ws = w_s.seeds_to_w(G, seeds, truncation_psi=0.7)
    with torch.no_grad():
        ws_o = Go.mapping(synthetic.seed_latents(seeds), None, truncation_psi=0.7)
    np.testing.assert_allclose(ws.cpu().numpy(), ws_o.numpy(), rtol=1e-4, atol=1e-4 * ws_o.abs().max().item())
    s = w_s.w_to_s(G, ws)
    s_o, _ = OS.get_styles(Go, ws_o)
    assert s.shape == (3, 26, 512)
    np.testing.assert_allclose(s.cpu().numpy(), s_o.numpy(), rtol=1e-4, atol=1e-4 * s_o.abs().max().item())


@pytest.mark.parametrize("use_whitelist", [False, True])
def test_generate_fromS_mapper_vs_oracle(use_whitelist):
    """--use_mapper 1 (generate_fromS.py:117-122,149-165): per-item direction from the latent mapper."""
    from stylemc_amd import generate_fromS, utils
    from stylemc_amd.latent_mappers import Mapper
    G, Go = _pair(32, 512)
    m = Mapper(neg_slope=0.01).eval()
    m.load_state_dict(synthetic.seeded_state_dict(m, seed=8))
    styles = synthetic.synthetic_styles(3, seed=4)
    got = list(generate_fromS.render_pairs(G, styles.to(DEV), None, 3.0, utils.get_temp_shapes(G),
                                           mapper=m.to(DEV), use_whitelist=use_whitelist))
    ref = OG.render_pairs(Go, styles.clone(), None, 3.0, OS.get_temp_shapes(Go), mapper=m.cpu(),
                          use_whitelist=use_whitelist)
    for (i, imgs), rimgs in zip(got, ref):
        for k in range(2):
            _check_u8(imgs[k], rimgs[k], f"item {i} power {k}")


def test_generate_fromS_projected_w_vs_oracle():
    """--projected-w (generate_fromS.py:89-102): G.synthesis(w) for each W row, uint8 per-pixel."""
    from stylemc_amd import generate_fromS, w_s
    G, Go = _pair(1024, 32768)
    ws = w_s.seeds_to_w(G, [5, 6], truncation_psi=0.7)
    got = [img for _, img in generate_fromS.render_projected_w(G, ws)]
    ref = OG.render_projected_w(Go, ws.cpu())
    for a, b in zip(got, ref):
        _check_u8(a, b, "projected w")


def test_generate_fromS_config5_video_sweep_64_frames():
    """BASELINE config 5: the FFHQ-1024 --from_video sweep, change_power 0 -> 50, 64 frames rendered on the GPU in
    batches of 8; frames {0, 21, 42, 63} checked per pixel against the oracle (the uint8 tolerance above)."""
    from stylemc_amd import generate_fromS, utils
    G, Go = _pair(1024, 32768)
    style_row = synthetic.synthetic_styles(1, seed=3)[0]
    direction = torch.zeros(1, 26, 512)
    direction[:, utils.S_TRAINABLE_SPACE_CHANNELS] = torch.randn(1, 8, 512, generator=torch.Generator().manual_seed(2)) * 0.1
    powers = np.linspace(0.0, 50.0, 64)
    got = generate_fromS.render_sweep(G, style_row.to(DEV), direction.to(DEV), powers, utils.get_temp_shapes(G),
                                      batch=8)
    assert got.shape == (64, 1024, 1024, 3)
    idx = [0, 21, 42, 63]
    ref = OG.render_sweep(Go, style_row, direction, powers[idx], OS.get_temp_shapes(Go))
    _check_u8(got[idx], ref, "config 5 sweep")
    # the frames differ along the sweep (the direction is applied)
    assert (got[0].int() - got[63].int()).abs().float().mean() > 1.0


def _second_generator(res, cbase, seed):
    from stylemc_amd import networks
    cfg = synthetic.generator_config(resolution=res, channel_base=cbase)
    sd = synthetic.generator_state_dict(cfg, seed=seed)
    G2 = networks.build_generator(cfg, sd, device=DEV)
    Go2 = ON.Generator(512, 0, 512, res, 3, channel_base=cbase, conv_clamp=cfg["conv_clamp"])
    Go2.load_state_dict(sd, strict=False)
    return G2, Go2.eval().requires_grad_(False)


@pytest.mark.parametrize("res,cbase", [(32, 512), (256, 16384)])
def test_generate_fromS_network2_vs_oracle(res, cbase):
    """--network2 (generate_fromS.py:80-86,168-170): the edited image from a second seeded generator, the original
    from the first; per-pixel vs the oracle, and the edited image differs from G's own rendering."""
    from stylemc_amd import generate_fromS, utils
    G, Go = _pair(res, cbase)
    G2, Go2 = _second_generator(res, cbase, seed=1)
    styles = synthetic.synthetic_styles(2, seed=9)
    direction = torch.zeros(1, 26, 512)
    direction[:, utils.S_TRAINABLE_SPACE_CHANNELS] = torch.randn(1, 8, 512, generator=torch.Generator().manual_seed(1)) * 0.3
    ts, ts2 = utils.get_temp_shapes(G), utils.get_temp_shapes(G2)   # (get_temp_shapes replaces the affines)
    tso, tso2 = OS.get_temp_shapes(Go), OS.get_temp_shapes(Go2)
    got = list(generate_fromS.render_pairs(G, styles.to(DEV), direction.to(DEV), 2.0, ts, G2=G2, temp_shapes2=ts2))
    ref = OG.render_pairs(Go, styles.clone(), direction, 2.0, tso, G2=Go2, temp_shapes2=tso2)
    one = list(generate_fromS.render_pairs(G, styles.to(DEV), direction.to(DEV), 2.0, ts))
    for (i, imgs), rimgs, (_, single) in zip(got, ref, one):
        for k in range(2):
            _check_u8(imgs[k], rimgs[k], f"item {i} power {k}")
        assert torch.equal(imgs[0], single[0])
        assert not torch.equal(imgs[1], single[1])
    # video sweep: power-0 frames from G, the rest from G2
    powers = [0.0, 1.0, 2.0]
    frames = generate_fromS.render_sweep(G, styles[0].to(DEV), direction.to(DEV), powers, ts, batch=2, G2=G2,
                                         temp_shapes2=ts2)
    ref0 = OG.render_sweep(Go, styles[0], direction, powers[:1], tso)
    ref12 = OG.render_sweep(Go2, styles[0], direction, powers[1:], tso2)
    _check_u8(frames[:1], ref0, "sweep G frame")
    _check_u8(frames[1:], ref12, "sweep G2 frames")
