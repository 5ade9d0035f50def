#!/bin/bash
# TEMP A/B of row-kernel variants (SMC_ROWV): correctness of the 3x3 shapes, then the layer-set timing.
OUT=gpurun_out/${1:-rowab}; mkdir -p $OUT
for v in ${VARIANTS:-9 0 1 2 3}; do
  SMC_ROWV=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread -k same3x3 > $OUT/pytest_$v.log 2>&1
  rc=$?; echo "variant $v pytest rc=$rc $(tail -1 $OUT/pytest_$v.log)"; case $rc in 0) ;; 1) continue;; *) exit $rc;; esac
  SMC_ROWV=$v timeout -k 10 300 python tools/bench_gemm.py --reps 10 > $OUT/bench_$v.txt 2>&1 || exit 1
  grep -E "conv1  r=  (128|256|512)|conv1  r= 1024|TOTAL" $OUT/bench_$v.txt | sed "s/^/v$v /"
done
