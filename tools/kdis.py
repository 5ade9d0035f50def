"""Disassembly of the gfx950 kernels of a built library whose symbol contains a pattern.

    python tools/kdis.py [lib.so] pattern > out.s
"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def main():
    lib = sys.argv[1] if len(sys.argv) > 2 else "stylemc_amd/_lib/libstylemc_hip.so"
    pat = sys.argv[-1]
    with tempfile.TemporaryDirectory() as d:
        shutil.copy(lib, os.path.join(d, "lib.so"))
        subprocess.run([OBJDUMP, "--offloading", "lib.so"], cwd=d, check=True, capture_output=True)
        for b in sorted(f for f in os.listdir(d) if f.endswith("gfx950")):
            t = subprocess.run([OBJDUMP, "-d", os.path.join(d, b)], check=True, capture_output=True, text=True).stdout
            cur = None
            for line in t.splitlines():
                m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
                if m:
                    cur = m.group(1)
                if cur and pat in cur:
                    print(line)


if __name__ == "__main__":
    main()
