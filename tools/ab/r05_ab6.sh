#!/bin/bash
# r05: split-bf16 wide tiles (256 output channels, conv_gemm_x3_kernel AS; base) vs without (nowide, SMC_X3_WIDE=0).
# Tests on the base library, per-layer GEMM times (tools/bench_gemm.py) for both, then interleaved bench rounds.
OUT=gpurun_out/${1:-r05_ab6}; ROUNDS=${2:-2}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "conv_gemm or synthesis_1024 or synthesis_layer" > $OUT/pytest_base.log 2>&1
rc=$?; echo "base tests rc=$rc: $(tail -1 $OUT/pytest_base.log)"; [ $rc -eq 0 ] || exit 1
for v in base nowide; do
  lib=stylemc_amd/_lib/libstylemc_hip.so; [ $v = base ] || lib=_lib_ab/$v/libstylemc_hip.so
  SMC_HIP_LIB=$lib timeout -k 10 300 python tools/bench_gemm.py > $OUT/gemm_$v.txt 2>&1 || { echo "gemm $v failed"; tail -5 $OUT/gemm_$v.txt; exit 1; }
  echo "gemm $v: $(grep -E 'conv0  r=  (128|256)' $OUT/gemm_$v.txt | tr -s ' ' | tr '\n' '|') $(grep TOTAL $OUT/gemm_$v.txt)"
done
run() {  # tag lib extra-args
  local tag=$1 lib=$2; shift 2
  SMC_HIP_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > $OUT/bench_${tag}_$r.log 2>&1
  local rc=$?; [ $rc -eq 0 ] || { echo "$tag bench rc=$rc"; tail -5 $OUT/bench_${tag}_$r.log; exit $rc; }
  python - $OUT/bench_${tag}_$r.log $tag <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
parts = {k: (v["ms_per_step"], v["frac"]) for k, v in d["roofline"]["parts"].items()}
print(sys.argv[2], d["value"], d["ms_per_step"], parts, flush=True)
PY
}
for r in $(seq 1 $ROUNDS); do
  run base stylemc_amd/_lib/libstylemc_hip.so
  run nowide _lib_ab/nowide/libstylemc_hip.so
done
