#!/bin/bash
# wino4 per-layer bench + PMC on the F(4x4) / F(2x2) r=64 and r=256 launches + loss-phase wall / trace.
OUT=gpurun_out/r03_p2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u -m pytest tests/test_gpu_wino4.py -x -q --timeout 100 --timeout-method thread > $OUT/pytest_w4.log 2>&1
rc=$?; tail -3 $OUT/pytest_w4.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/bench_wino.py --reps 10 > $OUT/bench_wino.txt 2>&1
rc=$?; cat $OUT/bench_wino.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u tools/loss_trace.py run 20 > $OUT/loss_wall.txt 2>&1
rc=$?; cat $OUT/loss_wall.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/losstr -o p --output-format csv -- python -u tools/loss_trace.py run 20 > $OUT/loss_prof.log 2>&1
rc=$?; [ $rc -ne 0 ] && { tail -20 $OUT/loss_prof.log; exit $rc; }
python tools/loss_trace.py analyze $(find $OUT/losstr -name '*kernel_trace.csv' | head -1) > $OUT/loss_gaps.txt 2>&1; cat $OUT/loss_gaps.txt
for spec in "fwd4 64" "bwd4 64" "fwd 64" "fwd4 256" "fwd 256"; do
  set -- $spec; tag=${1}_$2
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU -d $OUT/$tag.a -o p --output-format csv -- python tools/wino_one.py $1 $2 > $OUT/$tag.a.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS -d $OUT/$tag.b -o p --output-format csv -- python tools/wino_one.py $1 $2 > $OUT/$tag.b.log 2>&1 || exit 1
done
echo PROBE2_DONE
