#!/bin/bash
# split-bf16 direct convs: tests of both product forms, then the bench with x3 and fp32 conv products
OUT=gpurun_out/${1:-r04_x3}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_find_direction.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -4 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for cp in x3 fp32 x3 fp32; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --conv-products $cp > $OUT/bench_$cp.log 2>&1
  rc=$?; [ $rc -eq 0 ] || exit $rc
  python - $OUT/bench_$cp.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]; parts = {k: (v["ms_per_step"], v["frac"]) for k, v in r["parts"].items()}
print(d["config"]["conv_products"], d["value"], d["ms_per_step"], parts)
PY
done
