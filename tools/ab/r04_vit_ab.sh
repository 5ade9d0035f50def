#!/bin/bash
# ViT split-bf16 GEMMs: tower tests of both forms, then bench A/B (vit x3 / fp32, Winograd tile cap 64 variant)
OUT=gpurun_out/${1:-r04_vit}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_vit.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_vit.log 2>&1
rc=$?; tail -3 $OUT/pytest_vit.log
[ $rc -eq 0 ] || exit $rc
run() {  # tag lib args...
  tag=$1; lib=$2; shift 2
  SMC_HIP_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > $OUT/$tag.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$tag rc=$rc"; tail -5 $OUT/$tag.log; exit $rc; }
  python - $OUT/$tag.log $tag <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]; parts = {k: (v["ms_per_step"], v["frac"]) for k, v in r["parts"].items()}
print(sys.argv[2], d["value"], d["ms_per_step"], parts, flush=True)
PY
}
B=stylemc_amd/_lib/libstylemc_hip.so
for r in 1 2; do
  run base_$r $B
  run vitfp32_$r $B --vit-products fp32
  run tc64_$r _lib_ab/tc64/libstylemc_hip.so
done
