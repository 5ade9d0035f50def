#!/bin/bash
# r06: PMC passes over tools/bench_blur.py (the conv0 FIR forward at the FFHQ-1024 batch-4 shapes): HBM bytes, L2 hits,
# wave-state buckets.  One counter set per pass.
OUT=gpurun_out/${1:-r06/blur_pmc}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/a -o p --output-format csv -- python tools/bench_blur.py > $OUT/a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d $OUT/b -o p --output-format csv -- python tools/bench_blur.py > $OUT/b.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS -d $OUT/c -o p --output-format csv -- python tools/bench_blur.py > $OUT/c.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $OUT/t -o p --output-format csv -- python tools/bench_blur.py > $OUT/t.log 2>&1 || exit 1
python tools/pmc_read.py "$OUT/a/p_counter_collection.csv" "$OUT/b/p_counter_collection.csv" "$OUT/c/p_counter_collection.csv" > $OUT/summary.txt 2>&1
grep -A20 blur_act_v4 $OUT/summary.txt
