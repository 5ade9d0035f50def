"""Exec-free network pickle loading (stylemc_amd.legacy).

No real StyleGAN2-ADA pickle exists offline, so the fixtures are built here with the reduce protocol of
torch_utils/persistence.py:119-127: every network module pickles as
``_reconstruct_persistent_obj(dict(type='class', version=6, module_src=..., class_name=..., state=__dict__))``
(tensors and parameters through torch's own reducers, storages as ``_load_from_bytes`` blobs), and the
top-level object is the dict legacy.py:21-61 expects.  The stored module source raises if executed, so a
successful load also proves nothing from the file ran."""
import collections
import io
import os
import pickle
import sys
import types

import numpy as np
import pytest
import torch

from stylemc_amd import legacy, networks, synthetic

EVIL_SRC = "raise RuntimeError('the pickled module source was executed')\n"


def _fake_persistence_module():
    """A stand-in `torch_utils.persistence` so pickle can *write* the persistent reduce by name."""
    mod = types.ModuleType("torch_utils.persistence")

    def _reconstruct_persistent_obj(meta):  # only referenced by name in the pickle stream
        raise AssertionError("never called while writing")

    _reconstruct_persistent_obj.__module__ = "torch_utils.persistence"
    _reconstruct_persistent_obj.__qualname__ = "_reconstruct_persistent_obj"
    mod._reconstruct_persistent_obj = _reconstruct_persistent_obj
    pkg = types.ModuleType("torch_utils")
    pkg.persistence = mod
    return pkg, mod


class _Persistent:
    def __init__(self, fn, class_name, state):
        self.fn, self.class_name, self.state = fn, class_name, state

    def __reduce__(self):
        meta = dict(type="class", version=6, module_src=EVIL_SRC, class_name=self.class_name, state=self.state)
        return self.fn, (meta,)


def _as_persistent(module, fn, init_kwargs=None):
    """persistence.py:119-127: the persistent object's state is the module's WHOLE __dict__ (hook
    OrderedDicts, _non_persistent_buffers_set, plain attributes, numpy scalars, ...)."""
    # (this package's own per-layer kernel caches are not part of an upstream layer's __dict__)
    state = {k: v for k, v in module.__dict__.items() if not type(v).__module__.startswith("stylemc_amd")}
    state["training"] = False
    state["_modules"] = collections.OrderedDict((k, _as_persistent(m, fn)) for k, m in module._modules.items()
                                                if m is not None)
    if init_kwargs is not None:
        state["_init_kwargs"] = init_kwargs
    return _Persistent(fn, type(module).__name__, state)


def _make_pickle(G, init_kwargs, extra=None, protocol=4):
    pkg, mod = _fake_persistence_module()
    saved = {k: sys.modules.get(k) for k in ("torch_utils", "torch_utils.persistence")}
    sys.modules["torch_utils"], sys.modules["torch_utils.persistence"] = pkg, mod
    try:
        fn = mod._reconstruct_persistent_obj
        top = dict(G=_as_persistent(G, fn, init_kwargs), D=_as_persistent(torch.nn.Linear(2, 2), fn),
                   G_ema=_as_persistent(G, fn, init_kwargs), training_set_kwargs=None, augment_pipe=None)
        if extra:
            top.update(extra)
        return pickle.dumps(top, protocol=protocol)
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v


def _generator(res=32, cbase=512):
    cfg = synthetic.generator_config(resolution=res, channel_base=cbase, conv_clamp=256)
    G = networks.build_generator(cfg, synthetic.generator_state_dict(cfg, seed=2), device="cpu")
    kw = dict(z_dim=512, c_dim=0, w_dim=512, img_resolution=res, img_channels=3,
              mapping_kwargs=dict(num_layers=8), synthesis_kwargs=dict(channel_base=cbase, channel_max=512,
                                                                        num_fp16_res=0, conv_clamp=256))
    return G, kw


@pytest.mark.parametrize("protocol", [2, 3, 4])
def test_roundtrip_state_and_config(tmp_path, protocol):
    """Protocol 3 is what the official pickles use (Python 3.7 default); 2 and 4 for completeness."""
    G, kw = _generator()
    G.synthesis.b8.conv1.weight_gain_np = np.float64(1 / 3)     # numpy scalars live in real __dict__s
    G.synthesis.b8.conv1.register_buffer("scratch", torch.zeros(2), persistent=False)
    assert G.synthesis.b8.conv1._non_persistent_buffers_set
    path = tmp_path / "net.pkl"
    blob = _make_pickle(G, kw, protocol=protocol)
    if protocol <= 3:
        assert b"set" in blob
    path.write_bytes(blob)
    G2 = legacy.load_generator_pkl(str(path), device="cpu")
    del G.synthesis.b8.conv1.scratch
    a, b = G.state_dict(), G2.state_dict()
    assert a.keys() == b.keys()
    for k in a:
        assert torch.equal(a[k], b[k]), k
    assert G2.img_resolution == 32 and G2.synthesis.block_resolutions == G.synthesis.block_resolutions


def test_load_generator_cli_path(tmp_path):
    from stylemc_amd.find_direction import load_generator
    G, kw = _generator()
    path = tmp_path / "net.pkl"
    path.write_bytes(_make_pickle(G, kw))
    from stylemc_amd.find_direction import until_k_for
    # --resolution selects the rendered depth (find_direction.py:263), not the generator: any value loads
    G2 = load_generator(str(path), 16, "cpu")
    assert torch.equal(G2.synthesis.b32.conv1.weight, G.synthesis.b32.conv1.weight)
    assert until_k_for(G2, 16) == 2 and until_k_for(G2, 32) == 3
    with pytest.raises(SystemExit):
        until_k_for(G2, 64)


class _Evil:
    def __init__(self, fn, args):
        self.fn, self.args = fn, args

    def __reduce__(self):
        return self.fn, self.args


@pytest.mark.parametrize("fn,args", [(os.system, ("echo pwned",)), (eval, ("1+1",)),
                                     (getattr, ("", "join"))])
def test_rejects_non_allow_listed_callables(fn, args):
    G, kw = _generator(res=8)
    blob = _make_pickle(G, kw, extra={"evil": _Evil(fn, args)})
    with pytest.raises(pickle.UnpicklingError):
        legacy.load_network_pkl(io.BytesIO(blob))


def test_rejects_non_module_reconstructor():
    blob = pickle.dumps(collections.Counter(a=1))  # a class outside the allow-list
    with pytest.raises(pickle.UnpicklingError):
        legacy.load_network_pkl(io.BytesIO(blob))


def test_not_a_network_pickle():
    with pytest.raises(ValueError):
        legacy.load_network_pkl(io.BytesIO(pickle.dumps({"x": 1})))
