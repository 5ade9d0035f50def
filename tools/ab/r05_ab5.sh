#!/bin/bash
# r05: FIR backward built-in taps (base) vs runtime taps for both FIR kernels (bwdold); IR-SE50 split-bf16 products
# (bench --irse-products x3) on the base library; split-bf16 WO = 1 tiles with 16-channel K steps (k16).  Tests first, then interleaved bench rounds.
OUT=gpurun_out/${1:-r05_ab5}; ROUNDS=${2:-2}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "blur or synthesis_1024 or synthesis_layer or act_bwd" > $OUT/pytest_base.log 2>&1
rc=$?; echo "base tests rc=$rc: $(tail -1 $OUT/pytest_base.log)"; [ $rc -eq 0 ] || exit 1
SMC_HIP_LIB=_lib_ab/k16/libstylemc_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "conv_gemm" > $OUT/pytest_k16.log 2>&1
rc=$?; echo "k16 tests rc=$rc: $(tail -1 $OUT/pytest_k16.log)"; [ $rc -eq 0 ] || exit 1
run() {  # tag lib extra-args
  local tag=$1 lib=$2; shift 2
  SMC_HIP_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > $OUT/bench_${tag}_$r.log 2>&1
  local rc=$?; [ $rc -eq 0 ] || { echo "$tag bench rc=$rc"; tail -5 $OUT/bench_${tag}_$r.log; exit $rc; }
  python - $OUT/bench_${tag}_$r.log $tag <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
parts = {k: (v["ms_per_step"], v["frac"]) for k, v in d["roofline"]["parts"].items()}
print(sys.argv[2], d["value"], d["ms_per_step"], d["config"].get("irse_products"), parts, flush=True)
PY
}
for r in $(seq 1 $ROUNDS); do
  run base stylemc_amd/_lib/libstylemc_hip.so
  run bwdold _lib_ab/bwdold/libstylemc_hip.so
  run irsex3 stylemc_amd/_lib/libstylemc_hip.so --irse-products x3
  run k16 _lib_ab/k16/libstylemc_hip.so
done
