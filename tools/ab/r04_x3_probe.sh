#!/bin/bash
# per-layer direct-conv timing (tools/bench_gemm.py): fp32 MFMA, split-bf16, and the split kernel's timing probes
OUT=gpurun_out/${1:-r04_x3_probe}
mkdir -p $OUT
B=stylemc_amd/_lib/libstylemc_hip.so
timeout -k 10 200 python tools/bench_gemm.py --fp32 > $OUT/fp32.txt 2>&1 || exit 1
for v in base p1 p2 p4 p7; do
  if [ $v = base ]; then lib=$B; else lib=_lib_ab/$v/libstylemc_hip.so; fi
  SMC_HIP_LIB=$lib timeout -k 10 200 python tools/bench_gemm.py > $OUT/$v.txt 2>&1 || { echo "$v failed"; tail -3 $OUT/$v.txt; exit 1; }
done
python - $OUT <<'PY'
import sys, os, re
out = sys.argv[1]
tabs = {}
for v in ["fp32", "base", "p1", "p2", "p4", "p7"]:
    rows = {}
    for l in open(os.path.join(out, v + ".txt")):
        m = re.match(r"(\w+)\s+r=\s*(\d+).*?([\d.]+) us", l)
        if m:
            rows[(m.group(1), int(m.group(2)))] = float(m.group(3))
    tabs[v] = rows
keys = list(tabs["fp32"])
print("layer".ljust(18) + "".join(v.rjust(9) for v in tabs))
for k in keys:
    print(f"{k[0]}:{k[1]}".ljust(18) + "".join(f"{tabs[v].get(k, float('nan')):9.1f}" for v in tabs))
for v in tabs:
    print(v, "total us", round(sum(tabs[v].values()), 1))
PY
