"""Host-side checks of the HIP ViT and IR-SE50 drop-ins (no GPU): the packed weight layout agrees with the library's,
the state_dict keeps the openai/CLIP ``visual.*`` keys, and CPU tensors are refused (no CPU fallback)."""
import ctypes

import pytest
import torch

from stylemc_amd import _hip, synthetic, vit_hip
from stylemc_amd.clip_model import VIT_CONFIGS, VisionTransformer


@pytest.mark.parametrize("name", ["ViT-B/32", "ViT-B/16"])
def test_packed_layout_matches_library(name):
    m = vit_hip.HipVisionTransformer(**VIT_CONFIGS[name])
    m.refresh()  # raises if the Python packing and smc_vit_packed_floats disagree
    assert m.packed.numel() == _hip.load().smc_vit_packed_floats(ctypes.byref(m.cfg))
    # the first segment is conv1.weight^T [3*p*p][width]
    w = m.tower.conv1.weight.reshape(768, -1)
    assert torch.equal(m.packed[: w.numel()].view(w.shape[1], 768), w.t())


def test_state_dict_keys_and_reload():
    ref = VisionTransformer(**VIT_CONFIGS["ViT-B/32"])
    sd = synthetic.seeded_state_dict(ref, seed=4)
    m = vit_hip.HipVisionTransformer(**VIT_CONFIGS["ViT-B/32"])
    m.load_state_dict(sd)
    assert sorted(m.state_dict()) == sorted(ref.state_dict())
    p0 = m.packed.clone()
    sd2 = {k: v + 1 for k, v in sd.items()}
    m.load_state_dict(sd2)
    assert not torch.equal(p0, m.packed)


def test_unsupported_config_and_cpu_refused():
    lib = _hip.load()
    bad = vit_hip.vit_config(width=96, layers=1, heads=2, patch=4, grid=2, out_dim=32)  # head dim 48
    assert lib.smc_vit_packed_floats(ctypes.byref(bad)) == -1
    m = vit_hip.HipVisionTransformer(input_resolution=64, patch_size=32, width=128, layers=1, heads=2, output_dim=32)
    m.refresh()
    with pytest.raises(RuntimeError):
        m(torch.zeros(1, 3, 64, 64))


def test_irse50_descriptor_builds_on_host():
    """IR-SE50 packing (BN folds, adjoint phases) builds without a GPU; the library accepts the net."""
    from stylemc_amd import irse_hip
    net = irse_hip.HipIRSE50()
    pk = net.packed_net()
    assert pk.net.n_units == 24 and pk.net.flat == 512 * 7 * 7 and pk.net.stem_cin == 16
    strides = [pk.units[k].stride for k in range(24)]
    assert strides == [2, 1, 1, 2, 1, 1, 1, 2] + [1] * 13 + [2, 1, 1]
    assert all(pk.units[k].c2_bwd_nphases == (4 if strides[k] == 2 else 1) for k in range(24))
    assert [pk.units[k].sc_conv for k in (0, 3, 7, 21)] == [0, 1, 1, 1]
    lib = _hip.load()
    assert lib.smc_irse_saved_floats(ctypes.byref(pk.net), 4) > 0
    assert lib.smc_irse_workspace_bytes(ctypes.byref(pk.net), 4) > 0
    with pytest.raises(RuntimeError):
        net(torch.zeros(1, 3, 112, 112))
