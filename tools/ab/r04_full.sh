#!/bin/bash
# The whole -m gpu suite, smoke(), then the default bench (the round-end driver's sequence).
OUT=gpurun_out/${1:-r04_full}
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=15 \
    > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -4 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; tail -2 $OUT/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > $OUT/bench.log 2>&1
rc=$?; tail -1 $OUT/bench.log | cut -c1-400
exit $rc
