#!/bin/bash
# FIR forward strip kernel: bit-identity tests, then an interleaved A/B of the strip height (base 4 blocks, v4 = one
# block per workgroup, 2, 8) on the step's shapes.
OUT=gpurun_out/r03_blur
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "blur" -x -q --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_libs.sh $OUT/ab 2 "ablib/blur_v4 ablib/blur_sb2 ablib/blur_sb8" -- python -u tools/bench_blur.py
for f in $OUT/ab/*_1.txt; do echo "== $f"; grep -v amdgpu.ids $f; done
