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
    assert lib.smc_abi_version() == 4
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


def test_wino_shape_support_without_gpu():
    """smc_conv3x3_wino_supported is host logic (no device call): every synthesis conv1 from 32 px up has a
    Winograd kernel; narrower, odd-width, non-multiple-of-8 / 32 channel and >= 2 GiB inputs do not."""
    lib = _hip.load()
    for r in (32, 64, 128, 256, 512, 1024):
        c = min(32768 // r, 512)
        assert lib.smc_conv3x3_wino_supported(4, c, c, r, r) == 1, r
    assert lib.smc_conv3x3_wino_supported(4, 512, 512, 16, 16) == 0      # w < 32
    assert lib.smc_conv3x3_wino_supported(1, 64, 64, 112, 112) == 0     # 56 tile columns: no 64/32/16 block divides
    assert lib.smc_conv3x3_wino_supported(1, 64, 64, 96, 96) == 1       # 48 tile columns -> 16-column blocks
    assert lib.smc_conv3x3_wino_supported(1, 64, 64, 66, 64) == 0       # 33 tile rows: no 4-row block divides
    assert lib.smc_conv3x3_wino_supported(1, 64, 64, 64, 34) == 0       # w % 4
    assert lib.smc_conv3x3_wino_supported(1, 12, 32, 64, 64) == 0       # cin % 8
    assert lib.smc_conv3x3_wino_supported(1, 32, 48, 64, 64) == 0       # cout % 32
    assert lib.smc_conv3x3_wino_supported(16, 512, 512, 256, 256) == 0  # input >= 2 GiB (32-bit buffer offsets)


def test_dd_workspace_queries_without_gpu():
    """The epilogue backward kernels take their dd partials from a caller-owned workspace (no allocation inside the
    library): the queries are host logic, and a call that needs partials but gets no workspace fails
    on the host before any launch."""
    import ctypes
    lib = _hip.load()
    # act backward: float4 path 1024 floats per workgroup, scalar 2048 -> partials only beyond two workgroups
    assert lib.smc_modconv_act_bwd_workspace_size(4, 512, 32, 32) == 0        # 1024 px: one workgroup per plane
    assert lib.smc_modconv_act_bwd_workspace_size(4, 64, 64, 64) == 0         # 4096 px: 1 (vec4) / 2 workgroups
    assert lib.smc_modconv_act_bwd_workspace_size(2, 8, 128, 128) == 4 * 16 * 8    # 16384 px: 4 (vec4) / 8 workgroups
    assert lib.smc_modconv_act_bwd_workspace_size(1, 1, 7, 9) == 0
    # FIR backward: 32 x 64 u tiles; t tiles over the (2h+1)-wide gradient
    assert lib.smc_modconv_blur_act_bwd_workspace_size(4, 512, 8, 8, 9, 9) == 0
    assert lib.smc_modconv_blur_act_bwd_workspace_size(2, 8, 128, 128, 129, 129) == 4 * 16 * (3 * 5)
    assert lib.smc_modconv_blur_act_bwd_workspace_size(0, 8, 128, 128, 129, 129) == 0
    epi = _hip.ConvEpilogue()
    epi.mode = _hip.EPI_MODACT
    fake = ctypes.c_void_p(256)
    rc = lib.smc_modconv_act_bwd_f32(fake, fake, fake, fake, 2, 8, 128, 128, ctypes.byref(epi), None, 0, None)
    assert rc == 1 and b"workspace" in lib.smc_last_error()
    rc = lib.smc_modconv_blur_act_bwd_f32(fake, fake, fake, fake, 2, 8, 128, 128, 129, 129, 0, fake, 4, 4, 2, 2, 4.0, 1,
                                          ctypes.byref(epi), fake, 16, None)
    assert rc == 1 and b"workspace" in lib.smc_last_error()
