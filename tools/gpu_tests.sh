#!/bin/bash
# One GPU call: the named test files first (verbose, fail fast), then optionally the whole -m gpu suite.
# usage: bash tools/gpu_tests.sh TAG "tests/a.py tests/b.py" [full]
TAG=${1:-t}; FIRST=$2; OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ -n "$FIRST" ]; then
  timeout -k 10 600 python -u -m pytest $FIRST -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/first.log 2>&1
  rc=$?; tail -30 $OUT/first.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "$3" = "full" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider --durations=10 > $OUT/full.log 2>&1
  rc=$?; tail -15 $OUT/full.log; exit $rc
fi
