#!/bin/bash
# r05: split-K planning of the two loss networks when they run beside each other: IR-SE50 executor GEMMs planned for
# 4 (base) / 2 (aux2) / 1 (aux1) workgroups per CU; ViT GEMMs planned for all / half the CUs (lin2); both halved
# (both2).  Tests first (base: the conv GEMMs incl. the wide tile; aux1 / lin2: IR-SE50 / ViT), then bench rounds.
OUT=gpurun_out/${1:-r05_ab7}; ROUNDS=${2:-2}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "conv_gemm" > $OUT/pytest_base.log 2>&1
rc=$?; echo "base tests rc=$rc: $(tail -1 $OUT/pytest_base.log)"; [ $rc -eq 0 ] || exit 1
SMC_HIP_LIB=_lib_ab/both2/libstylemc_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_irse.py tests/test_gpu_vit.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_both2.log 2>&1
rc=$?; echo "both2 tests rc=$rc: $(tail -1 $OUT/pytest_both2.log)"; [ $rc -eq 0 ] || exit 1
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
  run aux2 _lib_ab/aux2/libstylemc_hip.so
  run aux1 _lib_ab/aux1/libstylemc_hip.so
  run lin2 _lib_ab/lin2/libstylemc_hip.so
  run both2 _lib_ab/both2/libstylemc_hip.so
done
