#!/bin/bash
# ViT GEMM variants: parity of each _lib_ab/<v> build (tests/test_gpu_vit.py linear + tower tests), then interleaved
# timing (tools/bench_linear.py per shape, tools/bench_vit.py tower) of the base library and the variants
OUT=gpurun_out/${1:-r04_lin_ab}
shift
mkdir -p $OUT
for v in "$@"; do
  SMC_HIP_LIB=_lib_ab/$v/libstylemc_hip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 \
    --timeout-method thread -m gpu tests/test_gpu_vit.py -k "linear or vit_forward" > $OUT/pytest_$v.log 2>&1 \
    || { echo "$v parity FAILED"; tail -20 $OUT/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $OUT/pytest_$v.log)"
done
for r in 1 2; do
  for v in base "$@"; do
    if [ $v = base ]; then lib=stylemc_amd/_lib/libstylemc_hip.so; else lib=_lib_ab/$v/libstylemc_hip.so; fi
    SMC_HIP_LIB=$lib timeout -k 10 200 python tools/bench_linear.py 4 8 > $OUT/lin_${v}_$r.txt 2>&1 || { tail -5 $OUT/lin_${v}_$r.txt; exit 1; }
    SMC_HIP_LIB=$lib timeout -k 10 200 python tools/bench_vit.py 8 > $OUT/vit8_${v}_$r.txt 2>&1 || exit 1
    SMC_HIP_LIB=$lib timeout -k 10 200 python tools/bench_vit.py 4 > $OUT/vit4_${v}_$r.txt 2>&1 || exit 1
    echo "$v round $r: $(grep TOTAL $OUT/lin_${v}_$r.txt | sed 's/torch.*//' | tr '\n' ' ') | $(grep -h 'hip:' $OUT/vit8_${v}_$r.txt $OUT/vit4_${v}_$r.txt | sed 's/ViT-B.32//' | tr '\n' ' ')"
  done
done
