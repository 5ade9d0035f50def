"""HBM traffic per launch of the synthesis modconv GEMM family (conv_gemm_lds_kernel / conv_gemm_kernel /
convt_gemm_kernel, TAG 0) from two rocprofv3 --pmc passes.

    python tools/pmc_traffic.py FETCH.csv WRITE.csv > profiles/pmc_traffic.json

Correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE / WRITE_SIZE are KiB; on gfx950 FETCH_SIZE
reports exactly half of the bytes of a wide coalesced streaming read -> read bytes = 2 x FETCH_SIZE x 1024;
WRITE_SIZE is exact for 16-B streaming stores -> write bytes = WRITE_SIZE x 1024.  The GEMM's input
reads are 4-B buffer loads (uncalibrated width), so the figure is an estimate (the guide's caveat).
"""
import csv
import json
import sys
from collections import defaultdict


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
    def fam(n):
        return ("conv_gemm" in n or "convt_gemm_kernel" in n) and ", 1>(" not in n

    fam_r = [v for d, v in fetch.items() if fam(names[d])]
    fam_w = [v for d, v in write.items() if fam(names_w[d])]
    rd = 2 * 1024 * sum(fam_r) / max(len(fam_r), 1)
    wr = 1024 * sum(fam_w) / max(len(fam_w), 1)
    out = {"conv_gemm_bytes_per_launch": round(rd + wr),
           "read_bytes_per_launch": round(rd), "write_bytes_per_launch": round(wr),
           "launches": [len(fam_r), len(fam_w)],
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE separate passes over bench.py --steps 2 --warmup 1 "
                     "(+ its 2-step serialised roofline pass); "
                     "read = 2 x FETCH_SIZE KiB (gfx950 correction), write = WRITE_SIZE KiB"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
