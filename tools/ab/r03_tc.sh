#!/bin/bash
# F(2x2) tile width A/B: base (TC up to 64 tiles per row block) vs ablib/tc32 (TC <= 32: 2 tile rows per block).
OUT=gpurun_out/r03_tc
mkdir -p $OUT
bash tools/ab_libs.sh $OUT/k 2 "ablib/tc32" -- python -u tools/bench_wino.py --res 512 1024 128 || exit 1
for f in $OUT/k/*_1.txt; do echo "== $f"; grep -v amdgpu.ids $f; done
bash tools/ab_libs.sh $OUT/s 3 "ablib/tc32" -- python -u tools/sensitivity.py --variant default --steps 30
