#!/bin/bash
# wino4 (role-specialised waves): GPU tests, probe, per-layer bench vs F(2x2).
OUT=gpurun_out/r03_w4b
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_gpu_wino4.py -x -v -s --timeout 150 --timeout-method thread > $OUT/pytest_w4.log 2>&1
rc=$?; grep -E "max err|PASS|FAIL|Error|error" $OUT/pytest_w4.log | tail -30; tail -3 $OUT/pytest_w4.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 tools/probes/wino4_probe > $OUT/wino4_probe.txt 2>&1
rc=$?; cat $OUT/wino4_probe.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/bench_wino.py --reps 10 > $OUT/bench_wino.txt 2>&1
rc=$?; cat $OUT/bench_wino.txt; exit $rc
