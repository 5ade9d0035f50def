#!/bin/bash
# Separate rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) over a short bench run, then the traffic summary.
# usage: bash tools/pmc_bench.sh OUTDIR
OUT=${1:-gpurun_out/pmc_bench}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c -d $OUT/$c -o p --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timer > $OUT/$c.log 2>&1 || { echo "PMC $c FAILED"; tail -5 $OUT/$c.log; exit 1; }
done
python tools/pmc_traffic.py $OUT/FETCH_SIZE/p_counter_collection.csv $OUT/WRITE_SIZE/p_counter_collection.csv > $OUT/traffic.json && cat $OUT/traffic.json
