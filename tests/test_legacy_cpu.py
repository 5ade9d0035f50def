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


# ------------------------------------------------------------------------------------------- TensorFlow-era pickles
# tests/golden/tf_legacy.npz: the REFERENCE's legacy.convert_tf_generator (legacy.py:110-204) run on a seeded synthetic
# TF generator (tests/golden/make_golden.py gen_tf_legacy): its variables, static kwargs, and every converted parameter
# and buffer.  The TF pickles here are written with the protocol of dnnlib.tflib.network.Network.__getstate__.


def _tf_fixture(golden):
    import json
    fx = golden("tf_legacy.npz")
    kw = json.loads(str(fx["static_kwargs"]))
    comps = {c: [(str(n), fx[f"tf:{c}:{n}"]) for n in fx[f"tf_names:{c}"]] for c in ("", "mapping", "synthesis")}
    sd = {k[3:]: (str(v[0]), tuple(int(d) for d in v[1:])) for k, v in fx.items() if k.startswith("sd:")}
    return fx, kw, comps, sd


def _same(t, ref):
    """t (a tensor) equals the fixture entry: shape + sha256 of the float32 bytes."""
    import hashlib
    a = np.ascontiguousarray(t.detach().cpu().numpy().astype(np.float32))
    return a.shape == ref[1] and hashlib.sha256(a.tobytes()).hexdigest() == ref[0]


def _fake_tf_module():
    """`dnnlib.tflib.network.Network` for *writing* TF-era pickles: NEWOBJ + BUILD with the __getstate__ dict."""
    mod = types.ModuleType("dnnlib.tflib.network")

    class Network:
        def __init__(self, state):
            self._state = state

        def __getstate__(self):
            return self._state

    Network.__module__, Network.__qualname__ = "dnnlib.tflib.network", "Network"
    mod.Network = Network
    pkg, sub = types.ModuleType("dnnlib"), types.ModuleType("dnnlib.tflib")
    pkg.tflib, sub.network = sub, mod
    return {"dnnlib": pkg, "dnnlib.tflib": sub, "dnnlib.tflib.network": mod}, Network


def _tf_pickle(kw, comps, protocol=3):
    mods, Network = _fake_tf_module()
    saved = {k: sys.modules.get(k) for k in mods}
    sys.modules.update(mods)
    try:
        def net(name, static, variables, components):
            return Network(dict(version=4, name=name, static_kwargs=static, components=components,
                                build_module_src=EVIL_SRC, build_func_name="G_main", variables=variables))
        G = net("G", dict(kw), comps[""], {"mapping": net("G_mapping", {}, comps["mapping"], {}),
                                          "synthesis": net("G_synthesis", {}, comps["synthesis"], {})})
        D = net("D", {}, [("Output/weight", np.zeros((4, 1), np.float32))], {})
        return pickle.dumps((G, D, G), protocol=protocol)
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v


def _stub_tree(kw, comps):
    def net(static, variables, components):
        n = legacy.TFNetworkStub()
        n.__setstate__(dict(version=4, static_kwargs=static, variables=variables, components=components))
        return n
    return net(kw, comps[""], {"mapping": net({}, comps["mapping"], {}), "synthesis": net({}, comps["synthesis"], {})})


def test_convert_tf_generator_matches_reference(golden):
    """Every parameter and buffer of the converted generator equals the reference's conversion bit for bit (the
    Conv0_up flip, transposes, mod_bias + 1, noise indices)."""
    _, kw, comps, sd_ref = _tf_fixture(golden)
    conv = legacy.convert_tf_generator(_stub_tree(kw, comps))
    G = legacy.generator_from_tf(conv, device="cpu")
    got = dict(list(G.named_parameters()) + list(G.named_buffers()))
    assert got.keys() == sd_ref.keys()
    for k, v in sd_ref.items():
        assert _same(got[k], v), k
    assert G.img_resolution == 32 and G.synthesis.b32.conv1.weight.shape == (16, 16, 3, 3)


@pytest.mark.parametrize("protocol", [2, 3, 4])
def test_tf_pickle_load(golden, tmp_path, protocol):
    """A (G, D, Gs) TF-era pickle through the exec-free unpickler (legacy.py:24-30): G_ema converted, the stored
    build_module_src (raises if executed) never run; the CLI loader path renders from it."""
    from stylemc_amd.find_direction import load_generator
    _, kw, comps, sd_ref = _tf_fixture(golden)
    path = tmp_path / "tf.pkl"
    path.write_bytes(_tf_pickle(kw, comps, protocol))
    data = legacy.load_network_pkl(open(path, "rb"))
    assert isinstance(data["G_ema"], legacy.TFGenerator) and isinstance(data["D"], legacy.TFNetworkStub)
    assert data["training_set_kwargs"] is None and data["augment_pipe"] is None
    G = load_generator(str(path), 32, "cpu")
    for k, v in G.state_dict().items():
        assert _same(v, sd_ref[k]), k


def test_tf_converted_generator_oracle_image(golden):
    """The converted weights drive the oracle generator to the reference-converted generator's image (the fixture
    was rendered by the oracle layers on the reference's conversion)."""
    from oracle import networks as ON
    fx, kw, comps, _ = _tf_fixture(golden)
    conv = legacy.convert_tf_generator(_stub_tree(kw, comps))
    ik = dict(conv.init_kwargs)
    mk = ik.pop("mapping_kwargs")
    Go = ON.Generator(**{k: ik.pop(k) for k in ("z_dim", "c_dim", "w_dim", "img_resolution", "img_channels")},
                      mapping_kwargs=mk, **ik).eval()
    Go.load_state_dict(conv.state_dict, strict=False)
    with torch.no_grad():
        img = Go(torch.from_numpy(fx["z"]), None, truncation_psi=0.7, noise_mode="const")
    assert torch.equal(img, torch.from_numpy(fx["img"]))


def test_tf_kwargs_rejections():
    with pytest.raises(ValueError, match="Unknown TensorFlow kwarg"):
        legacy._tf_kwargs({"resolution": 32, "not_a_kwarg": 1})
    kw = legacy._tf_kwargs({"label_size": 10})
    with pytest.raises(NotImplementedError):
        legacy.tf_generator_kwargs(kw)
    stub = legacy.TFNetworkStub()
    stub.__setstate__(dict(version=3, static_kwargs={}, variables=[], components={}))
    with pytest.raises(ValueError, match="version too low"):
        legacy.convert_tf_generator(stub)
