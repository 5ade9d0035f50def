"""Where is the GPU idle during the timed steps?  From a rocprofv3 kernel trace: the union of all streams' kernel
intervals over a time window, the idle gaps between them, and which kernels follow / precede the gaps.

    python tools/idle_gaps.py run_kernel_trace.csv [--from MS] [--to MS]   (ms from the first kernel of the trace)
Without --from/--to the window is the busiest stretch: the first and last kernel of the longest run of 5-ms
windows that are at least 50 % busy (the bench's warm-up + timed steps; the roofline pass comes after a pause).
"""
import collections
import csv
import re
import sys


def name(r):
    n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", n)[:44]


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    t0 = int(rows[0]["Start_Timestamp"])
    iv = [(int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0, name(r)) for r in rows]
    if "--from" in sys.argv:
        lo = float(sys.argv[sys.argv.index("--from") + 1]) * 1e6
        hi = float(sys.argv[sys.argv.index("--to") + 1]) * 1e6
    else:
        W = 5_000_000
        end = max(e for _, e, _ in iv)
        busy = []
        for w0 in range(0, end, W):
            segs = sorted((max(s, w0), min(e, w0 + W)) for s, e, _ in iv if e > w0 and s < w0 + W)
            tot, cs, ce = 0, None, None
            for s, e in segs:
                if ce is None or s > ce:
                    tot += (ce - cs) if ce is not None else 0
                    cs, ce = s, e
                else:
                    ce = max(ce, e)
            tot += (ce - cs) if ce is not None else 0
            busy.append(tot / W >= 0.5)
        best, run, start = (0, 0), 0, 0
        for i, b in enumerate(busy + [False]):
            if b:
                run += 1
                if run == 1:
                    start = i
            else:
                if run > best[1] - best[0]:
                    best = (start, start + run)
                run = 0
        lo, hi = best[0] * W, best[1] * W
    sel = [x for x in iv if lo <= x[0] <= hi]
    cur = sel[0][1]
    idle, nxt, prv, cnt = 0, collections.Counter(), collections.Counter(), collections.Counter()
    for i in range(1, len(sel)):
        s, e, n = sel[i]
        if s > cur:
            idle += s - cur
            nxt[n] += s - cur
            cnt[n] += 1
            prv[sel[i - 1][2]] += s - cur
        cur = max(cur, e)
    span = sel[-1][1] - sel[0][0]
    print(f"window {lo / 1e6:.1f}-{hi / 1e6:.1f} ms: {len(sel)} kernels, span {span / 1e6:.2f} ms, idle {idle / 1e6:.2f} ms "
          f"({100 * idle / span:.1f} %)")
    print("idle before (next kernel):")
    for n, v in nxt.most_common(12):
        print(f"  {v / 1e6:7.3f} ms {cnt[n]:5d} gaps  {n}")
    print("idle after (previous kernel):")
    for n, v in prv.most_common(8):
        print(f"  {v / 1e6:7.3f} ms  {n}")


if __name__ == "__main__":
    main()
