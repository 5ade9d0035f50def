"""Group a rocprofv3 kernel trace by (kernel, grid, workgroup) over the last `frac` of launches:
    python tools/trace_grid.py run_kernel_trace.csv [iters] [top]"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    keys = [k for k in rows[0] if "Grid" in k or "Workgroup" in k]
    agg = collections.defaultdict(lambda: [0, 0])
    tot = 0
    for r in rows:
        name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:60]
        g = "x".join(r[k] for k in keys if "Grid" in k)
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        agg[(name, g)][0] += d
        agg[(name, g)][1] += 1
        tot += d
    print(f"total {tot / 1e6 / iters:.3f} ms/iter over {len(rows)} launches ({len(rows) / iters:.0f}/iter)")
    for (name, g), (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
        print(f"{t / 1e3 / iters:9.1f} us/iter {c / iters:6.1f} calls {t / c / 1e3:8.1f} us/call  grid {g:>18s}  {name}")


if __name__ == "__main__":
    main()
