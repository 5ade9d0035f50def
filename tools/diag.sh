#!/bin/bash
# Step diagnostics on the GPU box: phase split, aten ops by device time, rocprofv3 kernel stats of a short bench.
# usage: bash tools/diag.sh TAG
TAG=${1:-diag}; OUT=gpurun_out/$TAG; mkdir -p $OUT
stop() { case $1 in 0) return 0;; *) echo "step rc=$1: stopping"; exit $1;; esac; }
timeout -k 10 300 python tools/phase_times.py --steps 10 > $OUT/phase.txt 2>&1; stop $?
cat $OUT/phase.txt | tail -6
timeout -k 10 300 python tools/aten_ops.py > $OUT/aten.txt 2>&1; stop $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timer > $OUT/prof.log 2>&1; stop $?
python tools/prof_summary.py $OUT/prof/run_kernel_trace.csv --steps 7 > $OUT/summary.md
head -40 $OUT/summary.md
