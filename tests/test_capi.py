"""The C-ABI library builds, loads on a CPU-only host and exports exactly what include/*.h declares."""
import ctypes
import os
import re

import pytest

from stylemc_amd import _hip, build

HEADER = os.path.join(build.INCLUDE, "stylemc_hip.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(smc_[a-z0-9_]+)\s*\(", text)))


def test_library_builds():
    assert os.path.exists(build.build(verbose=False))


def test_exports_match_header():
    lib = ctypes.CDLL(build.LIB)
    syms = declared_symbols()
    assert syms, "no declarations parsed"
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in include/stylemc_hip.h but not exported"
    assert sorted(_hip.exported_symbols()) == syms, "ctypes signatures out of sync with the header"


def test_exports_are_only_the_abi():
    out = os.popen(f"nm -D --defined-only {build.LIB}").read().split("\n")
    exported = sorted({l.split()[-1] for l in out if " T " in l and l.split()[-1].startswith("smc_")})
    assert exported == declared_symbols()


def test_abi_version_and_errors_without_gpu():
    lib = _hip.load()
    assert lib.smc_abi_version() == 2
    # argument validation runs on the host: no GPU needed, must fail loudly with a message
    rc = lib.smc_upfirdn2d_f32(None, None, None, 1, 4, 4, 99, 99, 4, 4, 1, 1, 1, 1, 1, 1, 1, 1, 0, 1.0, None)
    assert rc == 1
    assert b"out shape" in lib.smc_last_error()
    rc = lib.smc_conv_gemm_f32(None, 1, 16, 4, 4, None, 32, 4, 4, None, 1, None, None, None, 0, None)
    assert rc == 1


def test_cpu_tensors_rejected():
    import torch
    from stylemc_amd.torch_utils.ops import bias_act, upfirdn2d
    x = torch.zeros(1, 2, 4, 4)
    with pytest.raises(RuntimeError):
        bias_act.bias_act(x, act="lrelu")
    with pytest.raises(RuntimeError):
        upfirdn2d.upsample2d(x, upfirdn2d.setup_filter([1, 3, 3, 1]))
