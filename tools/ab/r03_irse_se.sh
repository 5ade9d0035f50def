#!/bin/bash
# IR-SE50 fused SE kernels: parity tests + loss-phase wall time.
OUT=gpurun_out/r03_se
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_irse.py -x -v --timeout 150 --timeout-method thread > $OUT/pytest_irse.log 2>&1
rc=$?; tail -15 $OUT/pytest_irse.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u tools/loss_trace.py run 20 > $OUT/loss_wall.txt 2>&1
rc=$?; cat $OUT/loss_wall.txt; exit $rc
