#!/bin/bash
# r05 FIR forward A/B (next tile's loads under this tile's FIR + stores) : blur tests on both libraries,
# tools/bench_blur.py per layer (bit-identical y checksums), interleaved bench rounds.
OUT=gpurun_out/${1:-r05_ab3}; ROUNDS=${2:-2}; VARS=${3:-"_lib_ab/wgs4 _lib_ab/nostd"}
mkdir -p $OUT
libof() { if [ "$1" = "base" ]; then echo stylemc_amd/_lib/libstylemc_hip.so; else echo $1/libstylemc_hip.so; fi; }
for v in base $VARS; do
  tag=$(basename $v)
  SMC_HIP_LIB=$(libof $v) timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_wino.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "blur or synthesis_1024 or synthesis_layer or wino" > $OUT/pytest_$tag.log 2>&1
  rc=$?; echo "$tag tests rc=$rc: $(tail -1 $OUT/pytest_$tag.log)"; [ $rc -eq 0 ] || exit 1
done
for v in base $VARS; do
  tag=$(basename $v)
  SMC_HIP_LIB=$(libof $v) timeout -k 10 200 python tools/bench_blur.py > $OUT/blur_$tag.txt 2>&1 || { echo "$tag bench_blur failed"; tail -3 $OUT/blur_$tag.txt; exit 1; }
  echo "== $tag"; cat $OUT/blur_$tag.txt | grep -v amdgpu.ids
done
for r in $(seq 1 $ROUNDS); do
  for v in base $VARS; do
    tag=$(basename $v)
    SMC_HIP_LIB=$(libof $v) timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_${tag}_$r.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$tag bench rc=$rc"; tail -5 $OUT/bench_${tag}_$r.log; exit $rc; }
    python - $OUT/bench_${tag}_$r.log $tag <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
parts = {k: (v["ms_per_step"], v["frac"]) for k, v in d["roofline"]["parts"].items()}
print(sys.argv[2], d["value"], d["ms_per_step"], parts, flush=True)
PY
  done
done
