"""Network pickles without code execution.

The reference loads StyleGAN2-ADA pickles with ``legacy.load_network_pkl`` (legacy.py:21-61), whose
unpickler rebuilds every network class by ``exec``-ing the module source stored inside the pickle
(torch_utils/persistence.py:185-207 ``_reconstruct_persistent_obj`` -> ``_src_to_module``).  Here the
pickle is read by a restricted unpickler that resolves only an allow-list of reconstruction functions:

* ``torch_utils.persistence._reconstruct_persistent_obj`` -> :class:`PersistentStub` (keeps ``meta``:
  class name + the object's ``__dict__`` state; the stored ``module_src`` is never executed),
* ``copyreg._reconstructor`` for plain ``torch.nn`` modules -> :class:`ModuleStub` (state kept),
* tensor / storage / parameter rebuilders (``torch._utils._rebuild_tensor_v2``, ``_rebuild_parameter``;
  storages via ``torch.storage._load_from_bytes`` -> ``torch.load(..., weights_only=True)``),
* ``collections.OrderedDict``, ``dnnlib.util.EasyDict`` (-> dict), numpy scalars/arrays (safe
  rebuilders only).

Anything else (``os.system``, ``builtins.eval``, arbitrary classes) raises ``pickle.UnpicklingError``.
The G_ema stub is then flattened into a state_dict with the parameter names of legacy.py:172-203 and the
generator is rebuilt from its stored ``init_kwargs`` with :class:`stylemc_amd.networks.Generator`.

TensorFlow-era pickles (the official StyleGAN2 ``stylegan2-ffhq-config-f.pkl`` and friends): a tuple of three
``dnnlib.tflib.network.Network`` objects (G, D, Gs), legacy.py:24-30.  Each becomes a :class:`TFNetworkStub` holding
its pickled state (version, static_kwargs, variables, components; ``build_module_src`` is kept as text and never
executed) and ``convert_tf_generator`` restates legacy.py:110-204 on plain numpy arrays: the kwargs table, the
parameter-name table with its transposes, the ``Conv0_up`` / ``Skip`` 180-degree weight flips, ``mod_bias + 1``
and the ``noise{2 log2(r) - 5 / - 4}`` index arithmetic.  Pinned: tests/golden/tf_legacy.npz, the reference's own
``convert_tf_generator`` on a seeded synthetic TF generator (tests/test_legacy_cpu.py reproduces its every
parameter and buffer bit for bit).  D is not converted (no discriminator on this path).

Parity: the PyTorch format is restated from persistence.py:119-127,185-207 and legacy.py:21-61; no real
StyleGAN2-ADA pickle exists offline, so the round trip is tested on pickles built with the same reduce
protocol from the package's own generator (tests/test_legacy_cpu.py) -- "parity unpinned" against a
real ffhq.pkl.
"""
import collections
import io
import pickle

import numpy as np
import torch

try:  # numpy >= 2 moved the array rebuilders; pickles written by numpy 1.x name numpy.core.multiarray
    from numpy._core import multiarray as _np_ma
except ImportError:  # pragma: no cover
    from numpy.core import multiarray as _np_ma

_PERSISTENT = ("torch_utils.persistence", "_reconstruct_persistent_obj")


class PersistentStub:
    """A persistent network object from the pickle, not reconstructed: ``class_name`` and ``state``."""

    def __init__(self, meta):
        meta = dict(meta)
        self.class_name = meta.get("class_name")
        self.version = meta.get("version")
        self.state = dict(meta.get("state") or {})

    def __repr__(self):
        return f"PersistentStub({self.class_name})"


class ModuleStub:
    """A plain (non-persistent) torch module from the pickle, e.g. ``torch.nn.Identity``."""

    def __init__(self, qualname=""):
        self.class_name = qualname
        self.state = {}

    def __setstate__(self, state):
        self.state = dict(state or {})


class TFNetworkStub:
    """A ``dnnlib.tflib.network.Network`` from a TensorFlow-era pickle: its __getstate__ dict, nothing rebuilt."""

    def __init__(self, *args):
        self.state = {}

    def __setstate__(self, state):
        self.state = dict(state or {})

    def __getattr__(self, name):   # version, static_kwargs, variables, components, ... (legacy.py attribute access)
        if name == "state":
            raise AttributeError(name)
        try:
            return self.state[name]
        except KeyError:
            raise AttributeError(name) from None

    def __repr__(self):
        return f"TFNetworkStub({self.state.get('name')})"


class _ClassRef:
    """Stand-in for a class the pickle references through copyreg._reconstructor (never imported)."""

    def __init__(self, module, name):
        self.qualname = f"{module}.{name}"


def _reconstructor(cls, base, state):
    if cls is TFNetworkStub:
        return TFNetworkStub()
    if isinstance(cls, _ClassRef) and cls.qualname.startswith("torch.nn.modules."):
        return ModuleStub(cls.qualname)
    raise pickle.UnpicklingError(f"copyreg._reconstructor of {getattr(cls, 'qualname', cls)!r} is not allowed")


def _load_storage(b):
    return torch.load(io.BytesIO(b), map_location="cpu", weights_only=True)


def _rebuild_parameter(data, requires_grad, backward_hooks):
    return data


def _rebuild_parameter_with_state(data, requires_grad, backward_hooks, state):
    return data


def _codecs_encode(obj, encoding="utf-8", errors="strict"):
    """Protocol-2 bytes: _codecs.encode(latin-1 str, 'latin1') (only str -> bytes, nothing else)."""
    if not isinstance(obj, str):
        raise pickle.UnpicklingError("_codecs.encode of a non-str")
    return obj.encode(encoding, errors)


class SafeNetworkUnpickler(pickle.Unpickler):
    _ALLOWED = {
        _PERSISTENT: PersistentStub,
        ("copyreg", "_reconstructor"): _reconstructor,
        ("torch._utils", "_rebuild_tensor_v2"): torch._utils._rebuild_tensor_v2,
        ("torch._utils", "_rebuild_parameter"): _rebuild_parameter,
        ("torch._utils", "_rebuild_parameter_with_state"): _rebuild_parameter_with_state,
        ("torch.storage", "_load_from_bytes"): _load_storage,
        ("collections", "OrderedDict"): collections.OrderedDict,
        ("dnnlib.util", "EasyDict"): dict,
        ("builtins", "object"): object,
        # nn.Module.__dict__ holds _non_persistent_buffers_set: under pickle protocol <= 3 (the official
        # pickles: Python 3.7, default protocol 3) a set is a REDUCE of builtins.set; protocol 2 names the
        # Python 2 module and encodes bytes through _codecs.encode
        ("builtins", "set"): set,
        ("builtins", "frozenset"): frozenset,
        ("__builtin__", "set"): set,
        ("__builtin__", "frozenset"): frozenset,
        ("__builtin__", "object"): object,
        ("copy_reg", "_reconstructor"): _reconstructor,
        ("_codecs", "encode"): _codecs_encode,
        ("numpy", "dtype"): np.dtype,
        ("numpy.core.multiarray", "scalar"): _np_ma.scalar,
        ("numpy.core.multiarray", "_reconstruct"): _np_ma._reconstruct,
        ("numpy._core.multiarray", "scalar"): _np_ma.scalar,
        ("numpy._core.multiarray", "_reconstruct"): _np_ma._reconstruct,
        ("numpy", "ndarray"): np.ndarray,
        ("dnnlib.tflib.network", "Network"): TFNetworkStub,
    }

    def find_class(self, module, name):
        fn = self._ALLOWED.get((module, name))
        if fn is not None:
            return fn
        if module.startswith("torch.nn.modules."):
            return _ClassRef(module, name)          # only usable through _reconstructor
        if module == "torch" and name.endswith("Storage"):
            return getattr(torch, name)             # storage type tags used by _rebuild_tensor_v2 pickles
        raise pickle.UnpicklingError(f"network pickle references {module}.{name}: not on the allow-list "
                                     f"(loading never imports or executes code from the file)")

    def persistent_load(self, pid):
        raise pickle.UnpicklingError("persistent ids are not used by network pickles")


def load_network_pkl(f):
    """legacy.py:21-61 without exec: {'G': stub, 'D': stub, 'G_ema': stub, ...}.  A TensorFlow-era (G, D, Gs) triple
    is converted as legacy.py:24-30 does: G and G_ema become :class:`TFGenerator` (init kwargs + state_dict), D stays
    a TFNetworkStub."""
    data = SafeNetworkUnpickler(f).load()
    if isinstance(data, tuple) and len(data) == 3 and all(isinstance(net, TFNetworkStub) for net in data):
        tf_G, tf_D, tf_Gs = data
        data = dict(G=convert_tf_generator(tf_G), D=tf_D, G_ema=convert_tf_generator(tf_Gs))
    if not isinstance(data, dict) or "G_ema" not in data:
        raise ValueError("not a StyleGAN2-ADA network pickle (expected a dict with 'G_ema', or the (G, D, Gs) triple "
                         "of a TensorFlow-era pickle)")
    data.setdefault("training_set_kwargs", None)
    data.setdefault("augment_pipe", None)
    return data


# ------------------------------------------------------------------------------------------- TensorFlow-era


class TFGenerator:
    """A converted TF-era generator: the [upstream] Generator's init kwargs and its state_dict (numpy -> torch)."""

    def __init__(self, init_kwargs, state_dict):
        self.init_kwargs, self.state_dict = init_kwargs, state_dict

    def __repr__(self):
        return f"TFGenerator({self.init_kwargs.get('img_resolution')} px)"


def _tf_params(tf_net):
    """Every variable of the network tree by its '/'-joined path (legacy.py:76-85)."""
    out = {}

    def walk(prefix, net):
        for name, value in net.variables:
            out[prefix + name] = np.asarray(value)
        for name, comp in dict(net.components or {}).items():
            walk(prefix + name + "/", comp)

    walk("", tf_net)
    return out


def _tf_kwargs(static):
    """The [upstream] Generator kwargs from the TF static_kwargs (legacy.py:114-156: names, defaults, and the same
    rejection of unknown keys)."""
    known = set()

    def kw(name, default=None, none=None):
        known.add(name)
        v = static.get(name, default)
        return v if v is not None else none

    out = dict(
        z_dim=kw("latent_size", 512), c_dim=kw("label_size", 0), w_dim=kw("dlatent_size", 512),
        img_resolution=kw("resolution", 1024), img_channels=kw("num_channels", 3),
        mapping_kwargs=dict(num_layers=kw("mapping_layers", 8), embed_features=kw("label_fmaps", None),
                            layer_features=kw("mapping_fmaps", None), activation=kw("mapping_nonlinearity", "lrelu"),
                            lr_multiplier=kw("mapping_lrmul", 0.01), w_avg_beta=kw("w_avg_beta", 0.995, none=1)),
        synthesis_kwargs=dict(channel_base=kw("fmap_base", 16384) * 2, channel_max=kw("fmap_max", 512),
                              num_fp16_res=kw("num_fp16_res", 0), conv_clamp=kw("conv_clamp", None),
                              architecture=kw("architecture", "skip"), resample_filter=kw("resample_kernel", [1, 3, 3, 1]),
                              use_noise=kw("use_noise", True), activation=kw("nonlinearity", "lrelu")))
    for name in ("truncation_psi", "truncation_cutoff", "style_mixing_prob", "structure"):
        kw(name)
    unknown = sorted(set(static) - known)
    if unknown:
        raise ValueError(f"Unknown TensorFlow kwarg {unknown[0]!r}")
    return out


def _tf_rules(p, log2):
    """(regex over the converted module's parameter / buffer names, value from the TF params) -- legacy.py:172-203.
    TF stores conv weights [kh, kw, in, out] and FC weights [in, out]; the upsampling convs of the TF graph are
    transposed convolutions, hence the spatial flip of Conv0_up / Skip."""
    conv = lambda w: w.transpose(3, 2, 0, 1)
    flip = lambda w: w[::-1, ::-1].transpose(3, 2, 0, 1)
    return (
        (r"mapping\.w_avg", lambda: p["dlatent_avg"]),
        (r"mapping\.embed\.weight", lambda: p["mapping/LabelEmbed/weight"].T),
        (r"mapping\.embed\.bias", lambda: p["mapping/LabelEmbed/bias"]),
        (r"mapping\.fc(\d+)\.weight", lambda i: p[f"mapping/Dense{i}/weight"].T),
        (r"mapping\.fc(\d+)\.bias", lambda i: p[f"mapping/Dense{i}/bias"]),
        (r"synthesis\.b4\.const", lambda: p["synthesis/4x4/Const/const"][0]),
        (r"synthesis\.b4\.conv1\.weight", lambda: conv(p["synthesis/4x4/Conv/weight"])),
        (r"synthesis\.b4\.conv1\.bias", lambda: p["synthesis/4x4/Conv/bias"]),
        (r"synthesis\.b4\.conv1\.noise_const", lambda: p["synthesis/noise0"][0, 0]),
        (r"synthesis\.b4\.conv1\.noise_strength", lambda: p["synthesis/4x4/Conv/noise_strength"]),
        (r"synthesis\.b4\.conv1\.affine\.weight", lambda: p["synthesis/4x4/Conv/mod_weight"].T),
        (r"synthesis\.b4\.conv1\.affine\.bias", lambda: p["synthesis/4x4/Conv/mod_bias"] + 1),
        (r"synthesis\.b(\d+)\.conv0\.weight", lambda r: flip(p[f"synthesis/{r}x{r}/Conv0_up/weight"])),
        (r"synthesis\.b(\d+)\.conv0\.bias", lambda r: p[f"synthesis/{r}x{r}/Conv0_up/bias"]),
        (r"synthesis\.b(\d+)\.conv0\.noise_const", lambda r: p[f"synthesis/noise{log2(r) * 2 - 5}"][0, 0]),
        (r"synthesis\.b(\d+)\.conv0\.noise_strength", lambda r: p[f"synthesis/{r}x{r}/Conv0_up/noise_strength"]),
        (r"synthesis\.b(\d+)\.conv0\.affine\.weight", lambda r: p[f"synthesis/{r}x{r}/Conv0_up/mod_weight"].T),
        (r"synthesis\.b(\d+)\.conv0\.affine\.bias", lambda r: p[f"synthesis/{r}x{r}/Conv0_up/mod_bias"] + 1),
        (r"synthesis\.b(\d+)\.conv1\.weight", lambda r: conv(p[f"synthesis/{r}x{r}/Conv1/weight"])),
        (r"synthesis\.b(\d+)\.conv1\.bias", lambda r: p[f"synthesis/{r}x{r}/Conv1/bias"]),
        (r"synthesis\.b(\d+)\.conv1\.noise_const", lambda r: p[f"synthesis/noise{log2(r) * 2 - 4}"][0, 0]),
        (r"synthesis\.b(\d+)\.conv1\.noise_strength", lambda r: p[f"synthesis/{r}x{r}/Conv1/noise_strength"]),
        (r"synthesis\.b(\d+)\.conv1\.affine\.weight", lambda r: p[f"synthesis/{r}x{r}/Conv1/mod_weight"].T),
        (r"synthesis\.b(\d+)\.conv1\.affine\.bias", lambda r: p[f"synthesis/{r}x{r}/Conv1/mod_bias"] + 1),
        (r"synthesis\.b(\d+)\.torgb\.weight", lambda r: conv(p[f"synthesis/{r}x{r}/ToRGB/weight"])),
        (r"synthesis\.b(\d+)\.torgb\.bias", lambda r: p[f"synthesis/{r}x{r}/ToRGB/bias"]),
        (r"synthesis\.b(\d+)\.torgb\.affine\.weight", lambda r: p[f"synthesis/{r}x{r}/ToRGB/mod_weight"].T),
        (r"synthesis\.b(\d+)\.torgb\.affine\.bias", lambda r: p[f"synthesis/{r}x{r}/ToRGB/mod_bias"] + 1),
        (r"synthesis\.b(\d+)\.skip\.weight", lambda r: flip(p[f"synthesis/{r}x{r}/Skip/weight"])),
        (r".*\.resample_filter", None),
    )


def tf_generator_kwargs(kwargs):
    """The converted kwargs as stylemc_amd.networks.Generator arguments; configurations this build does not run
    (conditional mapping, a non-skip architecture, other activations) raise."""
    import copy
    kw = copy.deepcopy(kwargs)
    mk, sk = kw.pop("mapping_kwargs"), kw.pop("synthesis_kwargs")
    if kw["c_dim"] != 0 or mk.pop("embed_features") is not None:
        raise NotImplementedError("TF generator with labels: conditional mapping networks are not supported")
    if mk.pop("layer_features") not in (None, kw["w_dim"]) or mk.pop("activation") != "lrelu":
        raise NotImplementedError("TF generator: only the lrelu mapping network of w_dim features is supported")
    if sk["architecture"] != "skip":
        raise NotImplementedError(f"TF generator architecture {sk['architecture']!r}: only 'skip' is supported")
    sk["resample_filter"] = tuple(sk["resample_filter"])
    return dict(kw, mapping_kwargs=mk, **sk)


def convert_tf_generator(tf_G):
    """legacy.py:110-204 without TensorFlow or code execution: a TFNetworkStub tree -> :class:`TFGenerator`.  The
    converted tensors are the reference's exactly (numpy transposes / flips / +1 of the stored float32 arrays)."""
    import re
    from . import networks
    if (tf_G.version or 0) < 4:
        raise ValueError("TensorFlow pickle version too low")
    kwargs = _tf_kwargs(dict(tf_G.static_kwargs or {}))
    p = _tf_params(tf_G)
    for name in list(p):
        if re.fullmatch(r"ToRGB_lod(\d+)/(.*)", name):
            # legacy.py:160-165 would switch to the 'orig' architecture (and fails there, kwargs.synthesis.kwargs)
            raise NotImplementedError("TF generator with ToRGB_lod* (architecture 'orig') is not supported")
    gkw = tf_generator_kwargs(kwargs)
    G = networks.Generator(**gkw)
    rules = _tf_rules(p, lambda r: int(np.log2(int(r))))
    sd = {}
    for name, t in list(G.named_parameters()) + list(G.named_buffers()):
        for pat, fn in rules:
            m = re.fullmatch(pat, name)
            if m:
                break
        else:
            raise KeyError(f"TF generator conversion: no rule for {name} {list(t.shape)}")
        if fn is None:
            continue
        v = torch.from_numpy(np.array(fn(*m.groups()), dtype=np.float32))
        if tuple(v.shape) != tuple(t.shape):
            raise ValueError(f"TF generator conversion: {name} {list(v.shape)} vs {list(t.shape)}")
        sd[name] = v
    return TFGenerator(gkw, sd)


def _named_tensors(obj, prefix=""):
    """Flatten a stub tree into (name, tensor) like nn.Module.state_dict (parameters, then buffers)."""
    state = obj.state
    skip = set(state.get("_non_persistent_buffers_set") or ())   # not in state_dict (nn.Module semantics)
    for key in ("_parameters", "_buffers"):
        for name, t in (state.get(key) or {}).items():
            if t is not None and not (key == "_buffers" and name in skip):
                yield prefix + name, t
    for name, child in (state.get("_modules") or {}).items():
        if child is not None:
            yield from _named_tensors(child, prefix + name + ".")


def stub_state_dict(stub):
    return {k: v.detach().to(torch.float32) if v.is_floating_point() else v for k, v in _named_tensors(stub)}


def stub_init_kwargs(stub):
    kw = stub.state.get("_init_kwargs")
    if kw is None:
        raise ValueError(f"{stub!r} carries no init_kwargs (persistence.py:103-105)")
    return dict(kw)


_SYNTH_KEYS = {"channel_base", "channel_max", "num_fp16_res", "conv_clamp", "architecture", "resample_filter"}
_MAP_KEYS = {"num_layers", "lr_multiplier", "w_avg_beta"}


def generator_from_stub(stub, device="cuda"):
    """Rebuild G_ema as stylemc_amd.networks.Generator from the pickle's init_kwargs + tensors."""
    from . import networks
    kw = stub_init_kwargs(stub)
    syn = {k: v for k, v in dict(kw.get("synthesis_kwargs") or {}).items() if k in _SYNTH_KEYS}
    if "resample_filter" in syn:
        syn["resample_filter"] = tuple(syn["resample_filter"])
    mk = {k: v for k, v in dict(kw.get("mapping_kwargs") or {}).items() if k in _MAP_KEYS}
    G = networks.Generator(kw["z_dim"], kw.get("c_dim", 0), kw["w_dim"], kw["img_resolution"], kw.get("img_channels", 3),
                           mapping_kwargs=mk, **syn)
    res = G.load_state_dict(stub_state_dict(stub), strict=False)
    bad = [k for k in res.missing_keys if not k.endswith("resample_filter")]
    if bad or res.unexpected_keys:
        raise KeyError(f"network pickle / Generator mismatch: missing={bad} unexpected={res.unexpected_keys}")
    return G.eval().requires_grad_(False).to(device)


def generator_from_tf(conv, device="cuda"):
    """A converted TF-era generator (:class:`TFGenerator`) as stylemc_amd.networks.Generator."""
    from . import networks
    G = networks.Generator(**conv.init_kwargs)
    res = G.load_state_dict(conv.state_dict, strict=False)
    bad = [k for k in res.missing_keys if not k.endswith("resample_filter")]
    if bad or res.unexpected_keys:
        raise KeyError(f"TF generator / Generator mismatch: missing={bad} unexpected={res.unexpected_keys}")
    return G.eval().requires_grad_(False).to(device)


def load_generator_pkl(path, device="cuda", key="G_ema"):
    with open(path, "rb") as f:
        data = load_network_pkl(f)
    net = data[key]
    if isinstance(net, TFGenerator):
        return generator_from_tf(net, device=device)
    return generator_from_stub(net, device=device)
