"""Register / LDS / scratch metadata of the gfx950 kernels in a built library whose name contains a pattern.

    python tools/kmeta.py [lib.so] pattern
"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
READOBJ = "/opt/rocm/lib/llvm/bin/llvm-readobj"
KEYS = [".vgpr_count", ".agpr_count", ".sgpr_count", ".group_segment_fixed_size", ".private_segment_fixed_size",
        ".vgpr_spill_count"]


def main():
    lib = sys.argv[1] if len(sys.argv) > 2 else "stylemc_amd/_lib/libstylemc_hip.so"
    pat = sys.argv[-1]
    with tempfile.TemporaryDirectory() as d:
        shutil.copy(lib, os.path.join(d, "lib.so"))
        subprocess.run([OBJDUMP, "--offloading", "lib.so"], cwd=d, check=True, capture_output=True)
        for b in sorted(f for f in os.listdir(d) if f.endswith("gfx950")):
            t = subprocess.run([READOBJ, "--notes", os.path.join(d, b)], check=True, capture_output=True,
                               text=True).stdout
            for blk in re.split(r"\n\s+- \.", t):
                m = re.search(r"\.name:\s+(\S+)", blk)
                if m and pat in m.group(1) and ".vgpr_count" in blk:
                    vals = []
                    for k in KEYS:
                        v = re.search(re.escape(k) + r":\s+(\S+)", blk)
                        vals.append(f"{k[1:]}={v.group(1) if v else '-'}")
                    print(m.group(1), " ".join(vals))


if __name__ == "__main__":
    main()
