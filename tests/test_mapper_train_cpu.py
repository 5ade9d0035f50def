"""train_latent_mapper's host logic (stylemc_amd.train_latent_mapper.MapperTrainer: per-image delta through the
synthesis, sum-form losses, gradient through the mapper, Adam with the cosine lr, seeded batch picks) on the CPU
with the oracle's synthesis and losses, against the REFERENCE's own loop (tests/golden/make_golden.py
gen_mapper_train -> mapper_train.npz: train_latent_mapper.py:138-196 on BASELINE config 1's problem, batch 2,
4 iterations).  Tolerances: batch picks identical, loss terms rtol 1e-3, the first gradient's per-tensor norms
rtol 1e-3, the total parameter update (subsampled) cosine >= 0.999 and per-tensor norms rtol 1e-2 (Adam's first
steps are ~lr * sign(g), so elements whose gradient is at fp32 noise level may flip)."""
import numpy as np
import torch

from oracle import synthesis as OS
from stylemc_amd import synthetic
from stylemc_amd.latent_mappers import Mapper
from stylemc_amd.train_latent_mapper import MapperTrainer
from tests.fd_helpers import OracleCLIP, OracleID, oracle_generator, oracle_rows_synth
from tests.test_reference_pins_cpu import LOSS_TEXT
from tests.test_reference_pins_cpu import _irse, _visual

SUB = 61   # make_golden.MAPPER_SUBSAMPLE


def _flat(m):
    return torch.cat([p.detach().reshape(-1) for p in m.parameters()])


def test_mapper_trainer_vs_reference_loop(golden):
    fx = golden("mapper_train.npz")
    res, bs, n_epochs, seed = (int(v) for v in fx["meta"])
    lr, slope = (float(v) for v in fx["meta_f"])
    torch.set_num_threads(8)
    Go = oracle_generator(res, 16384, seed=0)
    ts = OS.get_temp_shapes(Go)
    m = Mapper(slope)
    m.load_state_dict(synthetic.seeded_state_dict(m, seed=8))
    assert [n for n, _ in m.named_parameters()] == list(fx["param_names"])
    start = _flat(m).clone()
    tr = MapperTrainer(Go, torch.from_numpy(fx["styles"]), [(OracleCLIP(_visual("ViT-B/32"),
                                                                        synthetic.text_direction(*LOSS_TEXT)), 1.0)],
                       OracleID(_irse()), m, resolution=res, batch_size=bs, learning_rate=lr, n_epochs=n_epochs,
                       seed=seed, temp_shapes=ts, synth_fn=oracle_rows_synth)
    log = fx["log"]
    assert tr.total_iterations == len(log) == 4
    grad0 = None
    for row in log:
        last = tr.step()
        if grad0 is None:
            grad0 = torch.cat([p.grad.detach().reshape(-1) for p in m.parameters()])
        assert last["batch"] == int(row[1])
        np.testing.assert_allclose(last["lr"], row[2], rtol=1e-12)
        p = last["parts"].numpy()
        np.testing.assert_allclose(p[[0, 1, 3]], row[[4, 5, 6]], rtol=1e-3, atol=1e-6)
        np.testing.assert_allclose(float(last["grad_norm"]), row[7], rtol=1e-3)
    sizes = [q.numel() for q in m.parameters()]
    bounds = np.concatenate([[0], np.cumsum(sizes)])
    gn = np.array([grad0[a:b].norm().item() for a, b in zip(bounds[:-1], bounds[1:])])
    np.testing.assert_allclose(gn, fx["grad0_norms"], rtol=1e-3)
    cos = torch.nn.functional.cosine_similarity(grad0[::SUB].double(), torch.from_numpy(fx["grad0_sub"]).double(), dim=0)
    assert cos >= 0.9999, cos
    upd = _flat(m) - start
    un = np.array([upd[a:b].norm().item() for a, b in zip(bounds[:-1], bounds[1:])])
    np.testing.assert_allclose(un, fx["update_norms"], rtol=1e-2)
    cos = torch.nn.functional.cosine_similarity(upd[::SUB].double(), torch.from_numpy(fx["update_sub"]).double(), dim=0)
    assert cos >= 0.999, cos
