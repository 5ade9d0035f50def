"""HBM traffic per launch of the synthesis conv family (tools/conv_family.py: the direct implicit-GEMM kernels and
the Winograd kernel, TAG 0) from two rocprofv3 --pmc passes.

    python tools/pmc_traffic.py FETCH.csv WRITE.csv > profiles/pmc_traffic.json

Correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE / WRITE_SIZE are KiB; on gfx950 FETCH_SIZE
reports exactly half of the bytes of a wide coalesced streaming read -> read bytes = 2 x FETCH_SIZE x 1024;
WRITE_SIZE is exact for 16-B streaming stores -> write bytes = WRITE_SIZE x 1024.  The GEMM's input
reads are 4-B buffer loads (uncalibrated width), so the figure is an estimate (the guide's caveat).
"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from conv_family import is_family, is_wino  # noqa: E402


def per_dispatch(path, counter):
    vals = defaultdict(float)
    names = {}
    for r in csv.DictReader(open(path)):
        if (r.get("Counter_Name") or "") != counter:
            continue
        d = r.get("Dispatch_Id")
        vals[d] += float(r["Counter_Value"])
        names[d] = r.get("Kernel_Name", "")
    return vals, names


def main():
    fetch, names = per_dispatch(sys.argv[1], "FETCH_SIZE")
    write, names_w = per_dispatch(sys.argv[2], "WRITE_SIZE")
    def avg(vals, names, pred, scale):
        sel = [v for d, v in vals.items() if pred(names[d])]
        return scale * 1024 * sum(sel) / max(len(sel), 1), len(sel)

    rd, nr = avg(fetch, names, is_family, 2)
    wr, nw = avg(write, names_w, is_family, 1)
    wrd, _ = avg(fetch, names, is_wino, 2)
    wwr, nwino = avg(write, names_w, is_wino, 1)
    out = {"conv_gemm_bytes_per_launch": round(rd + wr),
           "read_bytes_per_launch": round(rd), "write_bytes_per_launch": round(wr),
           "launches": [nr, nw],
           "wino_bytes_per_launch": round(wrd + wwr), "wino_launches": nwino,
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE separate passes over bench.py --steps 2 --warmup 1 "
                     "(+ its 2-step serialised roofline pass); "
                     "read = 2 x FETCH_SIZE KiB (gfx950 correction), write = WRITE_SIZE KiB"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
