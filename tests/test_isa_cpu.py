"""Static checks of the built gfx950 code objects (CPU only: llvm-objdump on the library's offload bundles).

Round 6 traced the pipelined step's run-to-run difference to the attention backward writing LDS through generic
pointers (a scratch-resident struct array): misaligned flat_store_dwordx4 into LDS that now and then lost a dword
while other streams' kernels shared the CU.  Every kernel of the library addresses LDS and global
memory through typed pointers, so no FLAT memory instruction may appear in any of them.
"""
import os
import re
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "stylemc_amd", "_lib", "libstylemc_hip.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def _device_disasm(tmp_path):
    if not os.path.exists(OBJDUMP):
        pytest.skip("llvm-objdump not present")
    from stylemc_amd import build
    build.build(verbose=False)
    lib = tmp_path / "lib.so"
    shutil.copy(LIB, lib)
    subprocess.run([OBJDUMP, "--offloading", str(lib)], cwd=tmp_path, check=True, capture_output=True)
    bundles = sorted(p for p in os.listdir(tmp_path) if p.endswith("gfx950"))
    assert bundles, "no gfx950 code object in the library"
    out = []
    for b in bundles:
        r = subprocess.run([OBJDUMP, "-d", str(tmp_path / b)], check=True, capture_output=True, text=True)
        out.append(r.stdout)
    return "\n".join(out)


def _per_kernel(text, pattern):
    hits, cur = {}, None
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            cur = m.group(1)
            continue
        if cur and re.search(pattern, line):
            hits[cur] = hits.get(cur, 0) + 1
    return hits


def test_no_flat_memory_instructions(tmp_path):
    text = _device_disasm(tmp_path)
    assert "attn_bwd_kernel" in text, "attention backward kernel not found in the disassembly"
    flat = _per_kernel(text, r"\bflat_(load|store|atomic)")
    assert not flat, f"kernels with FLAT memory instructions (generic pointers): {flat}"
