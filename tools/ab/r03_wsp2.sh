#!/bin/bash
OUT=gpurun_out/r03_wsp2
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_wino_sp.py tests/test_gpu_irse.py -x -q --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_libs.sh $OUT/ab 2 "ablib/wg1" -- python -u tools/loss_trace.py run 20
grep irse $OUT/ab/*.txt
