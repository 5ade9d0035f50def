"""Cross-check bench.py's live roofline (HIP events around every smc_conv_gemm_f32 call of the serialised
roofline pass) against the rocprofv3 kernel trace of the same run.

    python tools/roofline_check.py run_kernel_trace.csv [launches=100]

The roofline pass is the last `launches` synthesis-GEMM calls of the run.  One smc_conv_gemm_f32 call is
the GEMM kernel (TAG 0) plus, where the layer needs them, the per-sample weight kernel (wscale_kernel, or
x3_weights_kernel for the split-bf16 planes) launched right before
it (wscale_kernel) and the split-K reduction launched right after it (epilogue_kernel); the HIP events
bracket all of them, so both the kernel-only and the whole-call averages are printed."""
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from conv_family import is_family  # noqa: E402


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    is_fam = lambda r: is_family(r["Kernel_Name"])
    idx = [i for i, r in enumerate(rows) if is_fam(r)][-n:]
    dur = lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    k_tot = sum(dur(rows[i]) for i in idx)
    call_tot = 0
    for i in idx:
        s, st = rows[i], rows[i]["Stream_Id"]
        start, end = int(s["Start_Timestamp"]), int(s["End_Timestamp"])
        j = i - 1
        while j >= 0 and rows[j]["Stream_Id"] != st:
            j -= 1
        if j >= 0 and any(k in rows[j]["Kernel_Name"] for k in ("wscale_kernel", "xscale_kernel", "x3_weights_kernel")):
            start = int(rows[j]["Start_Timestamp"])
        j = i + 1
        while j < len(rows) and rows[j]["Stream_Id"] != st:
            j += 1
        if j < len(rows) and "epilogue_kernel(" in rows[j]["Kernel_Name"] and "lin_" not in rows[j]["Kernel_Name"]:
            end = int(rows[j]["End_Timestamp"])
        call_tot += end - start
    print(f"last {len(idx)} synthesis GEMM launches (serialised roofline pass): kernel-only average "
          f"{k_tot / len(idx) / 1e3:.1f} us, whole smc_conv_gemm_f32 call (wscale + GEMM + split-K reduce, "
          f"first start to last end) {call_tot / len(idx) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
