#!/bin/bash
# r05: the tightened x3-vs-exact-fp32 conv tests, the end-to-end x3/fp32 direction test, the IR-SE50 conditioning
# diagnostic, and the default bench line.
OUT=gpurun_out/r05_x3acc; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_find_direction.py -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider -k "conv_gemm or x3_vs or identical_steps" > $OUT/pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL|x3 vs fp32|Error|assert" $OUT/pytest.log | tail -40; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u tools/irse_x3_diag.py > $OUT/irse_diag.txt 2>&1 || { tail -5 $OUT/irse_diag.txt; exit 1; }
cat $OUT/irse_diag.txt
timeout -k 10 400 python bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | cut -c1-300
