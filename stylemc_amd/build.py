"""Build the gfx950 kernel library (``stylemc_amd/_lib/libstylemc_hip.so``) with hipcc.

    python -m stylemc_amd.build [--force]

Each ``csrc/*.hip`` is compiled to an object (in parallel), then linked into one shared library
exporting exactly the C ABI of ``include/stylemc_hip.h`` (``-fvisibility=hidden`` + SMC_API).
Rebuilds only when a source/header is newer than the library.
"""
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(REPO, "include")
# A/B builds only (tools/): SMC_AB_OUT puts a variant library in its own directory, SMC_AB_DEFINES adds -D flags.
# The product build (no variables set) is the one stylemc_amd._hip loads.
OUT_DIR = os.environ.get("SMC_AB_OUT") or os.path.join(PKG, "_lib")
LIB = os.path.join(OUT_DIR, "libstylemc_hip.so")
AB_DEFINES = [f"-D{d}" for d in os.environ.get("SMC_AB_DEFINES", "").split()]
ARCH = os.environ.get("SMC_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", f"--offload-arch={ARCH}", "-I", INCLUDE,
          "-munsafe-fp-atomics", "-Wall", "-Wno-unused-function", "-Wno-unused-variable"]
# per-source extra flags: the Winograd kernel's transform runs beside its MFMAs, where packed f32 VALU (what the SLP
# vectorizer makes of adjacent scalar adds, plus the register moves that pair them) costs more than scalar ops
# (MI355X_MICROARCH.md 'price of one filler beside MFMAs'; tools/probes/wino_ab.hip: 3-5 % per launch)
FILE_FLAGS = {"wino.hip": ["-fno-slp-vectorize"], "wino4.hip": ["-fno-slp-vectorize"]}


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src):
    obj = os.path.join(OUT_DIR, os.path.basename(src)[:-4] + ".o")
    headers = glob.glob(os.path.join(CSRC, "*.hpp")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    if _stale(obj, [src] + headers):
        cmd = [HIPCC] + CFLAGS + AB_DEFINES + FILE_FLAGS.get(os.path.basename(src), []) + ["-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{r.stdout}\n{r.stderr}")
        if r.stderr.strip():
            print(r.stderr, file=sys.stderr)
    return obj


def build(force=False, verbose=True):
    os.makedirs(OUT_DIR, exist_ok=True)
    srcs = sources()
    headers = glob.glob(os.path.join(CSRC, "*.hpp")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    if not force and not _stale(LIB, srcs + headers + [os.path.abspath(__file__)]):
        return LIB
    if force:
        for o in glob.glob(os.path.join(OUT_DIR, "*.o")):
            os.remove(o)
    workers = max(1, min(len(srcs), int(os.environ.get("MAX_JOBS", "8"))))
    with cf.ThreadPoolExecutor(workers) as ex:
        objs = list(ex.map(_compile, srcs))
    tmp = LIB + ".tmp"
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, LIB)
    if verbose:
        print(f"built {LIB}")
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
