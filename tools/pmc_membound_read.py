"""Per-kernel summary of tools/pmc_membound.sh: HBM read (2 x FETCH_SIZE KiB, the gfx950 correction) and write
(WRITE_SIZE KiB) bytes per dispatch, the kernel's duration from the --kernel-trace pass (same command), achieved
HBM GB/s vs the 8 TB/s peak, VALU instructions per wave.   python tools/pmc_membound_read.py OUTDIR"""
import collections
import csv
import sys


def per_dispatch(path):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for r in csv.DictReader(open(path)):
        key = int(r["Dispatch_Id"])
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        meta[key] = (r["Kernel_Name"], int(r["Grid_Size"]))
    return per, meta


def main():
    out = sys.argv[1]
    merged = collections.defaultdict(lambda: collections.defaultdict(list))
    for tag in ("sq", "fetch", "write"):
        per, meta = per_dispatch(f"{out}/{tag}/p_counter_collection.csv")
        for d, v in per.items():
            for c, x in v.items():
                merged[meta[d]][c].append(x)
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(f"{out}/t/p_kernel_trace.csv")):
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        dur[(r["Kernel_Name"], grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"{'kernel':70s} {'grid':>9s} {'us':>7s} {'read MB':>8s} {'write MB':>8s} {'GB/s':>6s} {'frac':>5s} {'VALU/wave':>9s}")
    for (name, grid), v in sorted(merged.items()):
        if name.startswith(("void at::", "__amd")):
            continue
        mean = {c: sum(x) / len(x) for c, x in v.items()}
        ds = dur.get((name, grid))
        if not ds:
            continue
        us = sorted(ds)[len(ds) // 2]
        rd = 2 * mean.get("FETCH_SIZE", 0) * 1024
        wr = mean.get("WRITE_SIZE", 0) * 1024
        gbs = (rd + wr) / us / 1e3
        print(f"{name[:70]:70s} {grid:9d} {us:7.1f} {rd / 1e6:8.1f} {wr / 1e6:8.1f} {gbs:6.0f} {gbs / 8000:5.2f} "
              f"{mean.get('SQ_INSTS_VALU', 0) / max(mean.get('SQ_WAVES', 1), 1):9.0f}")


if __name__ == "__main__":
    main()
