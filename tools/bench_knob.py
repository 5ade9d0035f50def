"""bench.py with module switches set first (A/B of Python-side knobs, e.g. modconv.WINO4_MIN_CIN=64).
    python tools/bench_knob.py stylemc_amd.modconv.WINO4_MIN_CIN=64 [...] -- [bench.py args]"""
import ast
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if __name__ == "__main__":
    argv = sys.argv[1:]
    cut = argv.index("--") if "--" in argv else len(argv)
    for kv in argv[:cut]:
        k, v = kv.split("=", 1)
        mod, attr = k.rsplit(".", 1)
        setattr(importlib.import_module(mod), attr, ast.literal_eval(v))
    sys.argv = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")] + argv[cut + 1:]
    import bench
    bench.main()
