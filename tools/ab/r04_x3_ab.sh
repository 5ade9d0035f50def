#!/bin/bash
# split-bf16 conv kernel variants (ring depth, 32-channel K steps on the narrow tiles): interleaved bench A/B
OUT=gpurun_out/${1:-r04_x3_ab}; ROUNDS=${2:-1}; shift 2
VARS=${@:-"_lib_ab/nst3 _lib_ab/nst4 _lib_ab/k32s _lib_ab/nst3k32s"}
mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for v in base $VARS; do
    if [ "$v" = "base" ]; then lib=stylemc_amd/_lib/libstylemc_hip.so; else lib=$v/libstylemc_hip.so; fi
    tag=$(basename $v)
    SMC_HIP_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/${tag}_$r.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$tag rc=$rc"; exit $rc; }
    python - $OUT/${tag}_$r.log $tag <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]; parts = {k: (v["ms_per_step"], v["frac"]) for k, v in r["parts"].items()}
print(sys.argv[2], d["value"], d["ms_per_step"], parts, flush=True)
PY
  done
done
