#!/bin/bash
# Standard GPU-box sequence: build -> gpu tests -> bench -> rocprofv3 kernel stats.
# usage: bash tools/gpu_check.sh TAG [tests|notests] [bench args...]
set -o pipefail
TAG=${1:-run}; shift
MODE=${1:-tests}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
python -m stylemc_amd.build > $OUT/build.log 2>&1 || { echo "BUILD FAILED"; tail -20 $OUT/build.log; exit 1; }
if [ "$MODE" = "tests" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q --timeout=600 --durations=8 -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
  rc=$?
  tail -3 $OUT/pytest_gpu.log
  grep -E "^E   " $OUT/pytest_gpu.log | head -10
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > $OUT/bench.log 2>&1 || { echo "BENCH FAILED"; tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('VALUE', d['value'], d['unit'], 'ms/step', d['ms_per_step'], 'roofline', d['roofline'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timer > $OUT/prof.log 2>&1 || { echo "PROF FAILED"; tail -5 $OUT/prof.log; exit 1; }
python tools/prof_summary.py $OUT/prof/run_kernel_trace.csv --steps 7 > $OUT/summary.md
head -30 $OUT/summary.md
