#!/bin/bash
# One GPU call: the whole -m gpu suite, then the default bench (optionally a rocprofv3 kernel-trace of a short bench).
# usage: bash tools/r03_gpu_full.sh TAG [tests|notests] [prof|noprof]
TAG=${1:-full}; T=${2:-tests}; P=${3:-noprof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "$T" = "tests" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=10 \
      > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -4 $OUT/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1
rc=$?; tail -1 $OUT/bench.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
if [ "$P" = "prof" ]; then
  cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python bench.py --steps 10 --warmup 3 \
      --no-cpu-baseline > $OUT/bench_prof.log 2>&1
  rc=$?; tail -1 $OUT/bench_prof.log | cut -c1-200
  exit $rc
fi
