#!/bin/bash
# End-of-round pass on one GPU box: full GPU test suite, smoke(), default bench (with cpu_baseline + parity),
# rocprofv3 kernel-trace stats of a short bench, PMC traffic.  usage: bash tools/round_final.sh TAG
set -o pipefail
TAG=${1:-final}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
bash tools/round_artifacts.sh $TAG/art
