#!/bin/bash
# One GPU call for round 4: selected -m gpu tests, the 2-rank rehearsal of bench.py's own launcher (gloo, both ranks
# on the one GPU), then the default 1-GPU bench.
# usage: bash tools/r04_gpu.sh TAG "PYTEST_SELECTION" [dist|nodist] [bench|nobench]
TAG=${1:-r04}; SEL=${2:-}; D=${3:-dist}; B=${4:-bench}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$SEL" ]; then
  timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 \
      > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -5 $OUT/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "$D" = "dist" ]; then
  SMC_SHARE_GPU=1 SMC_DIST_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --steps 10 --warmup 3 \
      > $OUT/bench_dist2.log 2>&1
  rc=$?; tail -1 $OUT/bench_dist2.log | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
fi
if [ "$B" = "bench" ]; then
  timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1
  rc=$?; tail -1 $OUT/bench.log | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
fi
