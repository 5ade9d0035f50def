#!/bin/bash
# r05: second round of the loss-network split A/B (r05_ab7): base, lin2 / lin4 (ViT GEMMs planned for 1/2, 1/4 of the
# CUs), on the tree with the one-batch attention staging (its tests + tower times first).  (IR-SE50 planned for 1 workgroup per CU, aux1, flipped a PReLU kink of test_irse50_vs_torch_fp64[1]: dropped.)
OUT=gpurun_out/${1:-r05_ab8}; ROUNDS=${2:-2}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_vit.py tests/test_gpu_clip_text.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_base.log 2>&1
rc=$?; echo "base tests rc=$rc: $(tail -1 $OUT/pytest_base.log)"; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python tools/bench_vit.py 4 > $OUT/vit4_base.txt 2>&1 && timeout -k 10 200 python tools/bench_vit.py 8 > $OUT/vit8_base.txt 2>&1 || exit 1
grep hip $OUT/vit4_base.txt $OUT/vit8_base.txt
SMC_HIP_LIB=_lib_ab/lin4/libstylemc_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_irse.py tests/test_gpu_vit.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_lin4.log 2>&1
rc=$?; echo "lin4 tests rc=$rc: $(tail -1 $OUT/pytest_lin4.log)"; [ $rc -eq 0 ] || exit 1
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
  run lin2 _lib_ab/lin2/libstylemc_hip.so
  run lin4 _lib_ab/lin4/libstylemc_hip.so
done
