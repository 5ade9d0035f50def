#!/bin/bash
# ViT GEMM with the transposed-B staging: tower tests on the base library, tower timing and step A/B vs _lib_ab/nobt
OUT=gpurun_out/${1:-r04_vit_bt}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_vit.py \
  tests/test_gpu_clip_text.py > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  for v in base nobt; do
    if [ $v = base ]; then lib=stylemc_amd/_lib/libstylemc_hip.so; else lib=_lib_ab/$v/libstylemc_hip.so; fi
    SMC_HIP_LIB=$lib timeout -k 10 200 python tools/bench_vit.py 8 > $OUT/vit8_${v}_$r.txt 2>&1 || exit 1
    SMC_HIP_LIB=$lib timeout -k 10 200 python tools/bench_vit.py 4 > $OUT/vit4_${v}_$r.txt 2>&1 || exit 1
    echo "$v round $r: $(grep -h 'hip:' $OUT/vit8_${v}_$r.txt $OUT/vit4_${v}_$r.txt | sed 's/ViT-B.32//' | tr '\n' ' ')"
  done
done
bash tools/r04_x3_ab.sh ${OUT#gpurun_out/}/step 2 _lib_ab/nobt
