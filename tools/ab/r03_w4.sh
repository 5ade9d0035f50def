#!/bin/bash
# F(4x4) Winograd: GPU tests, per-layer A/B vs F(2x2) and the direct GEMM, then the step-sensitivity runs.
OUT=gpurun_out/r03_w4
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_wino4.py tests/test_gpu_wino.py -x -v -s --timeout 120 \
    --timeout-method thread > $OUT/pytest_w4.log 2>&1
rc=$?; tail -25 $OUT/pytest_w4.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/bench_wino.py --reps 10 > $OUT/bench_wino.txt 2>&1
rc=$?; cat $OUT/bench_wino.txt; [ $rc -ne 0 ] && exit $rc
if [ "$1" = "sens" ]; then
  timeout -k 10 500 python -u tools/sensitivity.py --variants default,no_clip,no_irse,no_losses,no_prefetch --rounds 2 \
      --steps 10 > $OUT/sens.txt 2>&1
  rc=$?; cat $OUT/sens.txt; exit $rc
fi
