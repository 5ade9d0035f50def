#!/bin/bash
OUT=gpurun_out/r03_vit
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_vit.py -x -q --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_libs.sh $OUT/ab 2 "ablib/notmb" -- python -u tools/loss_trace.py run 20
grep clip $OUT/ab/*.txt
bash tools/ab_libs.sh $OUT/bv 1 "ablib/notmb" -- python -u tools/bench_vit.py 8
cat $OUT/bv/*.txt | grep -v amdgpu
