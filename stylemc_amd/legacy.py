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

Parity: the format is restated from persistence.py:119-127,185-207 and legacy.py:21-61; no real
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


class _ClassRef:
    """Stand-in for a class the pickle references through copyreg._reconstructor (never imported)."""

    def __init__(self, module, name):
        self.qualname = f"{module}.{name}"


def _reconstructor(cls, base, state):
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
    """legacy.py:21-61 without exec: {'G': stub, 'D': stub, 'G_ema': stub, ...} (TF pickles unsupported)."""
    data = SafeNetworkUnpickler(f).load()
    if not isinstance(data, dict) or "G_ema" not in data:
        raise ValueError("not a StyleGAN2-ADA network pickle (expected a dict with 'G_ema'; "
                         "TensorFlow-era pickles need the reference's convert_tf_generator)")
    return data


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


def load_generator_pkl(path, device="cuda", key="G_ema"):
    with open(path, "rb") as f:
        data = load_network_pkl(f)
    return generator_from_stub(data[key], device=device)
