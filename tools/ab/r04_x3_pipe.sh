#!/bin/bash
# x3 direct-conv chunk pipeline A/B: parity of the new kernel, then per-layer timing (tools/bench_gemm.py) of
# fp32 MFMA, the previous split kernel (_lib_ab/old), the pipelined one, and its no-DMA/no-split probe (_lib_ab/p7)
OUT=gpurun_out/${1:-r04_x3_pipe}
mkdir -p $OUT
B=stylemc_amd/_lib/libstylemc_hip.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py \
  -k "conv or gemm" > $OUT/pytest_ops.log 2>&1 || { tail -30 $OUT/pytest_ops.log; exit 1; }
tail -2 $OUT/pytest_ops.log
timeout -k 10 200 python tools/bench_gemm.py --fp32 > $OUT/fp32.txt 2>&1 || exit 1
for v in old new p7; do
  if [ $v = new ]; then lib=$B; else lib=_lib_ab/$v/libstylemc_hip.so; fi
  SMC_HIP_LIB=$lib timeout -k 10 200 python tools/bench_gemm.py > $OUT/$v.txt 2>&1 || { echo "$v failed"; tail -3 $OUT/$v.txt; exit 1; }
done
python - $OUT <<'PY'
import sys, os, re
out = sys.argv[1]
tabs = {}
for v in ["fp32", "old", "new", "p7"]:
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
