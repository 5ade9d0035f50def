#!/bin/bash
# Stream-schedule A/B of bench.py in one call (interleaved, 3 rounds).  usage: bash tools/sched_ab.sh TAG
TAG=${1:-sched}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for round in 1 2 3; do
  for sc in pair prefetch; do
    timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-kernel-timer --schedule $sc \
        > $OUT/bench_${sc}_$round.txt 2>&1 || exit 1
    echo "$sc $round $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_${sc}_$round.txt)"
  done
done
