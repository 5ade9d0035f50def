"""Summarise a rocprofv3 --kernel-trace run as markdown, per find_direction step.

    python tools/prof_summary.py gpurun_out/prof1/run_kernel_trace.csv --steps N > profiles/rXX_summary.md

Only kernels from the first synthesis GEMM launch on are counted (model construction before it -- weight
uploads, packing -- is not part of a step); N = the steps run from there (bench warm-up + timed + roofline steps).
Without --steps, N is inferred from the CLIP tower: every find_direction step runs the ViT patch permutation
twice (im2col in the forward of the [edited; original] batch, its inverse in the backward).
Reports the top kernels and the aggregate of the synthesis modconv GEMM family (conv_gemm_lds_kernel /
conv_gemm_kernel / conv_row_kernel / convt_gemm_kernel instantiations with TAG 0 -- the IR-SE50 executor's
launches of the same kernels carry TAG 1 and are reported separately), whose average launch duration
bench.py's HIP-event roofline pass must match.
"""
import csv
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from conv_family import FAMILY, is_family as _is_family  # noqa: E402


def is_family(name):  # TAG 0 and TAG 1 (reported separately below)
    return any(f in name for f in FAMILY)


def load_rows(path):
    """Kernel dispatches as dicts with the CSV trace's keys: from a --output-format csv kernel trace, or from the
    rocpd SQLite database rocprofv3 writes by default (ROCm 7.2: `<name>_results.db`, view `kernels`)."""
    if path.endswith(".db"):
        import sqlite3
        con = sqlite3.connect(path)
        return [{"Kernel_Name": n, "Start_Timestamp": a, "End_Timestamp": b}
                for n, a, b in con.execute("select name, start, end from kernels")]
    return list(csv.DictReader(open(path)))


def main():
    path = sys.argv[1]
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else None
    rows = load_rows(path)
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    first = next(i for i, r in enumerate(rows) if is_family(r["Kernel_Name"]))
    rows = rows[first:]
    how = "given"
    if steps is None:
        perm = sum(1 for r in rows if "patch_perm_kernel" in r["Kernel_Name"])
        if perm >= 2:
            steps, how = perm // 2, "inferred: ViT patch permutations / 2"
    tot, cnt = defaultdict(float), defaultdict(int)
    for r in rows:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        tot[r["Kernel_Name"]] += d
        cnt[r["Kernel_Name"]] += 1
    total = sum(tot.values())
    span = int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])
    per = f" = {total / 1e6 / steps:.2f} ms/step" if steps else ""
    print(f"# rocprofv3 kernel trace: `{path}`\n")
    print(f"steps in the trace: {steps} ({how})\n" if steps else "steps in the trace: unknown (pass --steps)\n")
    print(f"from the first synthesis GEMM on: {len(rows)} launches, GPU kernel time {total / 1e6:.2f} ms{per} "
          f"(summed over streams), wall span {span / 1e6:.2f} ms" + (f" = {span / 1e6 / steps:.2f} ms/step" if steps else ""))
    fam = {k: v for k, v in tot.items() if is_family(k) and ", 1>(" not in k}
    aux = {k: v for k, v in tot.items() if is_family(k) and ", 1>(" in k}
    fc, ac = sum(cnt[k] for k in fam), sum(cnt[k] for k in aux)
    ft, at = sum(fam.values()), sum(aux.values())
    if fc:
        print(f"\nsynthesis modconv GEMM family (TAG 0: {' / '.join(FAMILY)}): {fc} launches, {ft / 1e6:.2f} ms"
              + (f" ({ft / 1e6 / steps:.2f} ms/step)" if steps else "")
              + f", average {ft / fc / 1e3:.1f} us/launch, {100 * ft / total:.1f}% of GPU kernel time")
    if ac:
        print(f"IR-SE50 executor GEMMs (TAG 1): {ac} launches, {at / 1e6:.2f} ms, average {at / ac / 1e3:.1f} us/launch")
    print()
    print("| ms total | ms/step | % | calls | avg us | kernel |\n|---:|---:|---:|---:|---:|---|")
    for k in sorted(tot, key=lambda k: -tot[k])[:32]:
        name = k.replace("|", "/")
        if len(name) > 110:
            name = name[:107] + "..."
        ps = f"{tot[k] / 1e6 / steps:.3f}" if steps else ""
        print(f"| {tot[k] / 1e6:.2f} | {ps} | {100 * tot[k] / total:.2f} | {cnt[k]} | {tot[k] / cnt[k] / 1e3:.1f} | `{name}` |")


if __name__ == "__main__":
    main()
