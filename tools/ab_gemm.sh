#!/bin/bash
# In-call A/B of library builds (stylemc_amd/_lib/ab_*.so) on tools/bench_gemm.py layers, interleaved.
# usage: bash tools/ab_gemm.sh TAG "bench_gemm --only filter" [variants...]
TAG=${1:-abg}; ONLY=${2:-}; shift 2; VS=${@:-A B}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for round in 1 2; do
  for v in $VS; do
    SMC_HIP_LIB=stylemc_amd/_lib/ab_$v.so timeout -k 10 200 python tools/bench_gemm.py --reps 20 ${ONLY:+--only $ONLY} \
        > $OUT/gemm_${v}_$round.txt 2>&1 || exit 1
    echo "== $v$round"; grep -v amdgpu.ids $OUT/gemm_${v}_$round.txt
  done
done
