"""Per-kernel breakdown of one phase of a rocprofv3 kernel trace (phases split at > 20 ms idle gaps, as in
tools/loss_trace.py).   python tools/trace_groups.py trace.csv GROUP ITERS [TOP]"""
import collections
import csv
import re
import sys


def main():
    path, gi, iters = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 30
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r) for r in rows]
    groups, cur = [], [iv[0]]
    for a, b in zip(iv, iv[1:]):
        if b[0] - a[1] > 20e6:
            groups.append(cur)
            cur = []
        cur.append(b)
    groups.append(cur)
    g = groups[gi]
    agg = collections.defaultdict(lambda: [0, 0])
    for a, b, r in g:
        n = re.sub(r"\(.*", "", r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", ""))[:48]
        key = (n, r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
        agg[key][0] += b - a
        agg[key][1] += 1
    tot = sum(v[0] for v in agg.values())
    span = g[-1][1] - g[0][0]
    print(f"group {gi}: {len(g) / iters:.1f} launches/iter, kernel sum {tot / iters / 1e3:.1f} us/iter, "
          f"span {span / iters / 1e3:.1f} us/iter")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
        print(f"{v[0] / iters / 1e3:8.1f} us/it {v[1] / iters:6.1f} calls {v[0] / v[1] / 1e3:7.1f} us/call  {k}")


if __name__ == "__main__":
    main()
