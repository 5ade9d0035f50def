#!/bin/bash
# parity of the base library on the touched kernels' tests, then an interleaved step A/B (bench.py) vs _lib_ab/<v>
OUT=gpurun_out/${1:-r04_step_ab}; ROUNDS=${2:-2}; TESTS=$3; shift 3
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $TESTS > $OUT/pytest.log 2>&1 \
    || { tail -30 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
bash tools/r04_x3_ab.sh ${OUT#gpurun_out/} $ROUNDS "$@"
