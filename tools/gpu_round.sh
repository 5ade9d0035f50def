#!/bin/bash
# One GPU-box call: pytest -m gpu (optionally a -k filter), then optionally the default bench.
# usage: bash tools/gpu_round.sh TAG [pytest -k expr|all] [bench|nobench]
# Every GPU step has its own time limit; a fault / abort / segfault / timeout ends the script.
TAG=${1:-run}; K=${2:-all}; B=${3:-bench}
OUT=gpurun_out/$TAG
mkdir -p $OUT
stop_on_fault() {
  case $1 in 0|1) return 0;; *) echo "step rc=$1: stopping"; exit $1;; esac
}
if [ "$K" != "none" ]; then
  if [ "$K" = "all" ]; then KARG=(); else KARG=(-k "$K"); fi
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=15 \
      "${KARG[@]}" > $OUT/pytest_gpu.log 2>&1
  rc=$?
  tail -25 $OUT/pytest_gpu.log
  stop_on_fault $rc
  [ $rc -eq 0 ] || exit 1
fi
if [ "$B" = "bench" ]; then
  timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1
  rc=$?
  tail -2 $OUT/bench.log
  exit $rc
fi
