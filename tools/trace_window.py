"""Busy-time analysis of a rocprofv3 kernel trace over the timed steps of a bench run.

    python tools/trace_window.py gpurun_out/X/prof/run_kernel_trace.csv MARKER PER_STEP STEPS

The window starts after the (k*PER_STEP)-th-from-last launch of the kernel whose name contains MARKER
(k = STEPS) -- e.g. ``patch_perm_kernel 3 5`` for bench.py --steps 5 (three ViT patch permutations per
find_direction step) -- and ends at the last kernel.

Prints the window span, the union of busy intervals (GPU busy fraction), per-stream busy time and the
kernels ranked by time inside the window (per step when steps_in_window is given)."""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    marker = sys.argv[2]
    per_step = int(sys.argv[3])
    steps = int(sys.argv[4])
    rows = list(csv.DictReader(open(path)))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"]) for r in rows)
    t1 = max(e for _, e, _, _ in iv)
    marks = [e for s, e, n, _ in iv if marker in n]
    w0 = marks[-per_step * steps - 1]
    win = [(max(s, w0), e, n, st) for s, e, n, st in iv if e > w0]
    span = t1 - w0
    busy, cur_s, cur_e = 0, None, None
    for s, e, _, _ in sorted(win):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    print(f"window {span / 1e6:.2f} ms, union busy {busy / 1e6:.2f} ms ({100 * busy / span:.1f}%), "
          f"sum of kernels {sum(e - s for s, e, _, _ in win) / 1e6:.2f} ms; per step: span {span / 1e6 / steps:.2f} ms, "
          f"busy {busy / 1e6 / steps:.2f} ms")
    per_stream = collections.Counter()
    for s, e, _, st in win:
        per_stream[st] += e - s
    for st, t in per_stream.most_common():
        print(f"  stream {st}: {t / 1e6 / steps:.2f} ms/step")
    per_k = collections.Counter()
    cnt = collections.Counter()
    for s, e, n, _ in win:
        key = n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:100]
        per_k[key] += e - s
        cnt[key] += 1
    for k, t in per_k.most_common(int(sys.argv[5]) if len(sys.argv) > 5 else 25):
        print(f"  {t / 1e6 / steps:7.3f} ms/step  {cnt[k] / steps:6.1f} calls  {k}")


if __name__ == "__main__":
    main()
