#!/bin/bash
# F(2x2) split-K: GPU tests, then an interleaved A/B of the split target (base 512, none, 1024) on the full step.
OUT=gpurun_out/r03_wsplit
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_wino.py tests/test_gpu_find_direction.py -x -q --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_libs.sh $OUT/ab 3 "ablib/nosplit ablib/t1024" -- python -u tools/sensitivity.py --variant default --steps 30
