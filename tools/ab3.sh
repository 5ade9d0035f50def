#!/bin/bash
# In-call A/B/C of library builds (stylemc_amd/_lib/ab_{A,B,C}.so): per-layer GEMM, ViT and IR-SE50 timings and a
# short bench, interleaved A B C A B C so box-to-box drift cancels.   usage: bash tools/ab3.sh TAG
TAG=${1:-ab}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for round in 1 2; do
  for v in A B C; do
    L=stylemc_amd/_lib/ab_$v.so
    [ -f $L ] || continue
    SMC_HIP_LIB=$L timeout -k 10 200 python tools/bench_gemm.py > $OUT/gemm_${v}_$round.txt 2>&1 || exit 1
    SMC_HIP_LIB=$L timeout -k 10 100 python tools/bench_vit.py 8 > $OUT/vit_${v}_$round.txt 2>&1 || exit 1
    SMC_HIP_LIB=$L timeout -k 10 100 python tools/bench_irse.py 8 > $OUT/irse_${v}_$round.txt 2>&1 || exit 1
    SMC_HIP_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_${v}_$round.txt 2>&1 || exit 1
    echo "$v$round $(tail -1 $OUT/gemm_${v}_$round.txt) | $(grep 'hip:' $OUT/vit_${v}_$round.txt | cut -c1-60) | $(grep 'hip:' $OUT/irse_${v}_$round.txt | cut -c1-60) | $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_${v}_$round.txt)"
  done
done
