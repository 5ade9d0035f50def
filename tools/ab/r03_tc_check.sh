#!/bin/bash
# After switching the F(2x2) tile cap to 32: the Winograd / synthesis-path GPU tests, smoke, one bench line.
OUT=gpurun_out/r03_tc_check
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_wino.py tests/test_gpu_ops.py tests/test_gpu_find_direction.py tests/test_gpu_generate.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; tail -1 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 420 python bench.py > $OUT/bench.log 2>&1
rc=$?; grep '^{' $OUT/bench.log | cut -c1-200; exit $rc
