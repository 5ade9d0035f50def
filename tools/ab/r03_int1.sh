#!/bin/bash
# Integration check: F(4x4) in the synthesis for cin >= 128 + fused IR-SE50 SE kernels.
OUT=gpurun_out/r03_int1
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_irse.py tests/test_gpu_wino4.py tests/test_gpu_ops.py tests/test_gpu_find_direction.py tests/test_gpu_generate.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -15 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u tools/loss_trace.py run 20 > $OUT/loss_wall.txt 2>&1
rc=$?; cat $OUT/loss_wall.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1
rc=$?; tail -2 $OUT/bench.log | cut -c1-1500; exit $rc
