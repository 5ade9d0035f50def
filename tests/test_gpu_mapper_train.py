"""train_latent_mapper on the GPU (MapperTrainer on the HIP synthesis, HIP CLIP ViT-B/32 and HIP IR-SE50) against
the REFERENCE's own loop (mapper_train.npz, tests/golden/make_golden.py gen_mapper_train: train_latent_mapper.py
:138-196 on BASELINE config 1's problem, batch 2, 4 iterations of Adam with the cosine lr).

Tolerances: batch picks identical; loss terms rtol 1e-3 / atol 5e-4 (fp32 summation order in every conv, as
config 1's pin); first gradient's per-tensor norms rtol 2e-3 and subsampled cosine >= 0.999; the total parameter
update: subsampled cosine >= 0.999 and per-tensor norms rtol 2e-2 (Adam's first steps are ~lr * sign(g))."""
import numpy as np
import pytest
import torch

from stylemc_amd import synthetic
from tests.test_reference_pins_cpu import LOSS_TEXT

pytestmark = pytest.mark.gpu
DEV = "cuda"
SUB = 61


def _flat(m):
    return torch.cat([p.detach().reshape(-1) for p in m.parameters()])


def test_train_latent_mapper_vs_reference_loop(golden):
    from stylemc_amd import build, networks
    from stylemc_amd.clip_loss import CLIPLoss
    from stylemc_amd.id_loss import IDLoss
    from stylemc_amd.latent_mappers import Mapper
    from stylemc_amd.train_latent_mapper import MapperTrainer
    build.build(verbose=False)
    fx = golden("mapper_train.npz")
    res, bs, n_epochs, seed = (int(v) for v in fx["meta"])
    lr, slope = (float(v) for v in fx["meta_f"])
    cfg = synthetic.generator_config(resolution=res)
    G = networks.build_generator(cfg, synthetic.generator_state_dict(cfg, seed=0), device=DEV)
    m = Mapper(slope)
    m.load_state_dict(synthetic.seeded_state_dict(m, seed=8))
    m = m.to(DEV)
    start = _flat(m).clone()
    clip = CLIPLoss(DEV, text_features=synthetic.text_direction(*LOSS_TEXT), synthetic_weights=True, seed=4)
    tr = MapperTrainer(G, torch.from_numpy(fx["styles"]).to(DEV), [(clip, 1.0)],
                       IDLoss(device=DEV, weights=None, seed=3), m, resolution=res, batch_size=bs, learning_rate=lr,
                       n_epochs=n_epochs, seed=seed)
    grad0 = None
    for row in fx["log"]:
        last = tr.step()
        if grad0 is None:
            grad0 = torch.cat([p.grad.detach().reshape(-1) for p in m.parameters()]).cpu()
        assert last["batch"] == int(row[1])
        p = last["parts"].cpu().numpy()
        np.testing.assert_allclose(p[[0, 1, 3]], row[[4, 5, 6]], rtol=1e-3, atol=5e-4)
    sizes = [q.numel() for q in m.parameters()]
    bounds = np.concatenate([[0], np.cumsum(sizes)])
    gn = np.array([grad0[a:b].norm().item() for a, b in zip(bounds[:-1], bounds[1:])])
    np.testing.assert_allclose(gn, fx["grad0_norms"], rtol=2e-3)
    cos = torch.nn.functional.cosine_similarity(grad0[::SUB].double(), torch.from_numpy(fx["grad0_sub"]).double(), dim=0)
    assert cos >= 0.999, cos
    upd = (_flat(m) - start).cpu()
    un = np.array([upd[a:b].norm().item() for a, b in zip(bounds[:-1], bounds[1:])])
    np.testing.assert_allclose(un, fx["update_norms"], rtol=2e-2)
    cos = torch.nn.functional.cosine_similarity(upd[::SUB].double(), torch.from_numpy(fx["update_sub"]).double(), dim=0)
    assert cos >= 0.999, cos


def test_train_latent_mapper_network2_vs_cpu_trainer():
    """--network2: the edited image from a second generator (train_latent_mapper.py:100-106,159-162).  GPU trainer
    vs the same MapperTrainer on the CPU with the oracle's synthesis and losses (pinned to the reference by
    test_mapper_train_cpu.py), 32-px generators G (seed 0) and G2 (seed 1), batch 2, 2 iterations."""
    from oracle import synthesis as OS
    from stylemc_amd import build, networks
    from stylemc_amd.clip_loss import CLIPLoss
    from stylemc_amd.id_loss import IDLoss
    from stylemc_amd.latent_mappers import Mapper
    from stylemc_amd.train_latent_mapper import MapperTrainer
    from tests.fd_helpers import OracleCLIP, OracleID, oracle_generator, oracle_rows_synth
    from tests.test_reference_pins_cpu import _irse, _visual
    build.build(verbose=False)
    text = synthetic.text_direction(*LOSS_TEXT)
    styles = synthetic.synthetic_styles(4, seed=6)
    cfg = synthetic.generator_config(resolution=32, channel_base=512)
    runs = []
    for dev in ("cpu", DEV):
        m = Mapper(0.01)
        m.load_state_dict(synthetic.seeded_state_dict(m, seed=8))
        if dev == "cpu":
            G, G2 = oracle_generator(32, 512, seed=0), oracle_generator(32, 512, seed=1)
            kw = dict(temp_shapes=OS.get_temp_shapes(G), temp_shapes2=OS.get_temp_shapes(G2), synth_fn=oracle_rows_synth)
            clip, idl = OracleCLIP(_visual("ViT-B/32"), text), OracleID(_irse())
        else:
            m = m.to(DEV)
            G = networks.build_generator(cfg, synthetic.generator_state_dict(cfg, seed=0), device=DEV)
            G2 = networks.build_generator(cfg, synthetic.generator_state_dict(cfg, seed=1), device=DEV)
            kw = {}
            clip = CLIPLoss(DEV, text_features=text, synthetic_weights=True, seed=4)
            idl = IDLoss(device=DEV, weights=None, seed=3)
        tr = MapperTrainer(G, styles.to(dev), [(clip, 1.0)], idl, m, resolution=32, batch_size=2, learning_rate=5e-4,
                           n_epochs=2, seed=1, G2=G2, **kw)
        parts = [tr.step()["parts"].cpu() for _ in range(2)]
        runs.append((parts, _flat(m).cpu()))
    (pc, wc), (pg, wg) = runs
    for a, b in zip(pg, pc):
        assert torch.allclose(a, b, rtol=1e-3, atol=5e-4), (a, b)
    m0 = Mapper(0.01)
    m0.load_state_dict(synthetic.seeded_state_dict(m0, seed=8))
    w0 = _flat(m0)
    cos = torch.nn.functional.cosine_similarity((wg - w0).double(), (wc - w0).double(), dim=0)
    assert cos >= 0.999, cos


def test_train_latent_mapper_cli(tmp_path):
    """The CLI drop-in (train_latent_mapper.py flags): a synthetic run with --network2 as a state_dict file writes
    mapper_<prompt>.pth, loadable into the Mapper (generate_fromS.py:117-122)."""
    import subprocess
    import sys
    cfg = synthetic.generator_config(resolution=256)
    g2 = tmp_path / "g2.pt"
    torch.save(synthetic.generator_state_dict(cfg, seed=1), g2)
    out = tmp_path / "run"
    r = subprocess.run([sys.executable, "-m", "stylemc_amd.train_latent_mapper", "--outdir", str(out),
                        "--text_prompt", "a b", "--clip_type", "small", "--resolution", "256", "--n_seeds", "4",
                        "--batch_size", "2", "--n_epochs", "1", "--network", "synthetic", "--network2", str(g2)],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "using 2 generators" in r.stdout
    from stylemc_amd.latent_mappers import Mapper
    m = Mapper(0.01)
    m.load_state_dict(torch.load(out / "mapper_a_b.pth", weights_only=True))
