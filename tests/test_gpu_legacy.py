"""A TensorFlow-era generator converted exec-free (stylemc_amd.legacy.convert_tf_generator) rendered on the HIP
synthesis: the image must match tests/golden/tf_legacy.npz, the reference-converted generator's image rendered by
the oracle layers (tests/golden/make_golden.py gen_tf_legacy).  Tolerance: 1e-4 of max |img| (the whole-network
image tolerance of tests/test_gpu_ops.py)."""
import pytest
import torch

from stylemc_amd import legacy
from tests.test_legacy_cpu import _stub_tree, _tf_fixture

pytestmark = pytest.mark.gpu


def test_tf_converted_generator_renders_vs_reference(golden):
    from stylemc_amd import build
    build.build(verbose=False)
    fx, kw, comps, _ = _tf_fixture(golden)
    G = legacy.generator_from_tf(legacy.convert_tf_generator(_stub_tree(kw, comps)), device="cuda")
    with torch.no_grad():
        img = G(torch.from_numpy(fx["z"]).cuda(), None, truncation_psi=0.7, noise_mode="const").cpu()
    ref = torch.from_numpy(fx["img"])
    assert torch.isfinite(img).all()
    err = (img - ref).abs().max().item()
    assert err <= 1e-4 * ref.abs().max().item(), err
