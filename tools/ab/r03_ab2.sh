#!/bin/bash
# A/B: CLIP-embedding prefetch (sensitivity variants) and the BK32 small-tile IR-SE50 GEMM (loss_trace).
OUT=gpurun_out/r03_ab2
mkdir -p $OUT
timeout -k 10 400 python -u tools/sensitivity.py --variants default,clip_pref --rounds 3 --steps 10 > $OUT/sens.txt 2>&1
rc=$?; cat $OUT/sens.txt; [ $rc -ne 0 ] && exit $rc
bash tools/ab_libs.sh $OUT/bk32 2 "ablib/bk32" -- python -u tools/loss_trace.py run 20
