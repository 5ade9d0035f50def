"""Aggregate rocprofv3 --pmc counter_collection.csv files: per kernel name, mean per dispatch of each counter."""
import csv
import glob
import sys
from collections import defaultdict


def load(path):
    per = defaultdict(lambda: defaultdict(list))
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        name = r.get("Kernel_Name") or r.get("KernelName") or r.get("Kernel-Name")
        cn = r.get("Counter_Name") or r.get("CounterName")
        v = float(r.get("Counter_Value") or r.get("CounterValue"))
        disp = r.get("Dispatch_Id") or r.get("Dispatch-Id") or r.get("DispatchId")
        per[name][(cn, disp)].append(v)
    out = defaultdict(dict)
    for name, d in per.items():
        acc = defaultdict(list)
        for (cn, disp), vals in d.items():
            acc[cn].append(sum(vals))  # sum over dimensions (XCDs / SEs) of one dispatch
        for cn, vals in acc.items():
            out[name][cn] = sum(vals) / len(vals)
    return out


if __name__ == "__main__":
    merged = defaultdict(dict)
    for pat in sys.argv[1:]:
        for path in glob.glob(pat):
            for k, v in load(path).items():
                merged[k].update(v)
    for k, v in merged.items():
        print(k[:100])
        for cn in sorted(v):
            print(f"   {cn:28s} {v[cn]:.4g}")
