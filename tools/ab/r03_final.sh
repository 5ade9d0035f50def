#!/bin/bash
# Final-tree GPU pass: the whole -m gpu suite, smoke(), then the round artefacts (bench with cpu_baseline, rocprof
# kernel stats, PMC traffic).  Stops at the first failure.
TAG=${1:-r03_final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=5 \
    > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; tail -2 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
bash tools/round_artifacts.sh ${TAG}_art
