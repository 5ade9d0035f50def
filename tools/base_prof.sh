#!/bin/bash
# One GPU call: the default bench line (no CPU leg), a rocprofv3 kernel-trace of a short bench summarised per step,
# and the loss-phase sensitivity.  usage: bash tools/base_prof.sh TAG [nosens]
set -o pipefail
TAG=${1:-base}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 400 python bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || { echo "BENCH FAILED"; tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 9 --warmup 2 --no-cpu-baseline > $OUT/prof_bench.log 2>&1 || { echo "PROF FAILED"; tail -5 $OUT/prof_bench.log; exit 1; }
python tools/prof_summary.py $OUT/prof/run_kernel_trace.csv > $OUT/kernel_stats.md
head -40 $OUT/kernel_stats.md
if [ "$2" != "nosens" ]; then
  timeout -k 10 400 python tools/sensitivity.py --variants default,no_clip,no_irse,no_losses > $OUT/sensitivity.txt 2>&1 || { echo "SENS FAILED"; tail -5 $OUT/sensitivity.txt; exit 1; }
  tail -6 $OUT/sensitivity.txt
fi
