"""Summarise a rocprofv3 --kernel-trace --stats run (kernel_stats.csv) as markdown.

    python tools/prof_summary.py gpurun_out/prof1/run_kernel_stats.csv [--steps N] > profiles/rXX_summary.md

Reports the top kernels and the aggregate of the conv_gemm_kernel family (all template
instantiations, plus the phase-fused convt_gemm_kernel that bench.py's timer also wraps), whose average launch duration bench.py's live HIP-event timing must match.
"""
import csv
import sys


def main():
    path = sys.argv[1]
    steps = None
    if "--steps" in sys.argv:
        steps = int(sys.argv[sys.argv.index("--steps") + 1])
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# rocprofv3 kernel stats: `{path}`\n")
    print(f"total GPU kernel time: {tot / 1e6:.2f} ms" + (f" over {steps} steps ({tot / 1e6 / steps:.2f} ms/step)" if steps else ""))
    fam = [r for r in rows if "conv_gemm_kernel" in r["Name"] or "convt_gemm_kernel" in r["Name"]]
    ft = sum(float(r["TotalDurationNs"]) for r in fam)
    fc = sum(int(r["Calls"]) for r in fam)
    if fc:
        print(f"\nconv_gemm_kernel family (incl. convt_gemm_kernel): {fc} launches, {ft / 1e6:.2f} ms, average {ft / fc / 1e3:.1f} us/launch, "
              f"{100 * ft / tot:.1f}% of GPU time\n")
    print("| ms total | % | calls | avg us | kernel |\n|---:|---:|---:|---:|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
        name = r["Name"].replace("|", "/")
        if len(name) > 110:
            name = name[:107] + "..."
        print(f"| {float(r['TotalDurationNs']) / 1e6:.2f} | {float(r['Percentage']):.2f} | {r['Calls']} | "
              f"{float(r['AverageNs']) / 1e3:.1f} | `{name}` |")


if __name__ == "__main__":
    main()
