#!/bin/bash
# One GPU call: a pytest -m gpu subset (-k expression) with its own time limit; stops on a fault / abort / timeout.
TAG=${1:-subset}; K=${2:-all}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "$K" = "all" ]; then KARG=(); else KARG=(-k "$K"); fi
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=20 \
    "${KARG[@]}" > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -30 $OUT/pytest_gpu.log
exit $rc
