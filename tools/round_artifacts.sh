#!/bin/bash
# One GPU-box pass that produces a round's measurement artefacts (then copy the summaries into profiles/):
#   default bench line (with cpu_baseline), rocprofv3 kernel-trace stats of the same bench, PMC traffic.
# usage: bash tools/round_artifacts.sh TAG
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 420 python bench.py > $OUT/bench.log 2>&1 || { echo "BENCH FAILED"; tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof_bench.log 2>&1 || { echo "PROF FAILED"; tail -5 $OUT/prof_bench.log; exit 1; }
python tools/prof_summary.py $OUT/prof/run_kernel_trace.csv > $OUT/kernel_stats.md
grep -o '"roofline.*' $OUT/prof_bench.log | cut -c1-300
head -8 $OUT/kernel_stats.md
bash tools/pmc_bench.sh $OUT/pmc > $OUT/pmc.log 2>&1 || { echo "PMC FAILED"; tail -5 $OUT/pmc.log; exit 1; }
cat $OUT/pmc/traffic.json
