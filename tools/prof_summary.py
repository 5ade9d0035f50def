"""Summarise a rocprofv3 --kernel-trace --stats run (kernel_stats.csv) as markdown.

    python tools/prof_summary.py gpurun_out/prof1/run_kernel_stats.csv [--steps N] > profiles/rXX_summary.md

Reports the top kernels and the aggregate of the synthesis modconv GEMM family (conv_gemm_lds_kernel /
conv_gemm_kernel / convt_gemm_kernel instantiations with TAG 0 -- the IR-SE50 executor's launches of the
same kernels carry TAG 1 and are reported separately), whose average launch duration bench.py's
HIP-event roofline pass must match.
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
    gemm = [r for r in rows if "conv_gemm" in r["Name"] or "convt_gemm_kernel" in r["Name"]]
    aux = [r for r in gemm if ", 1>(" in r["Name"]]
    fam = [r for r in gemm if r not in aux]
    at = sum(float(r["TotalDurationNs"]) for r in aux)
    ac = sum(int(r["Calls"]) for r in aux)
    ft = sum(float(r["TotalDurationNs"]) for r in fam)
    fc = sum(int(r["Calls"]) for r in fam)
    if fc:
        print(f"\nsynthesis modconv GEMM family (TAG 0: conv_gemm_lds_kernel / conv_gemm_kernel / convt_gemm_kernel): "
              f"{fc} launches, {ft / 1e6:.2f} ms, average {ft / fc / 1e3:.1f} us/launch, {100 * ft / tot:.1f}% of GPU time")
    if ac:
        print(f"IR-SE50 executor GEMMs (TAG 1): {ac} launches, {at / 1e6:.2f} ms, average {at / ac / 1e3:.1f} us/launch")
    print()
    print("| ms total | % | calls | avg us | kernel |\n|---:|---:|---:|---:|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
        name = r["Name"].replace("|", "/")
        if len(name) > 110:
            name = name[:107] + "..."
        print(f"| {float(r['TotalDurationNs']) / 1e6:.2f} | {float(r['Percentage']):.2f} | {r['Calls']} | "
              f"{float(r['AverageNs']) / 1e3:.1f} | `{name}` |")


if __name__ == "__main__":
    main()
