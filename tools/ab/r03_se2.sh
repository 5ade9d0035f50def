#!/bin/bash
OUT=gpurun_out/r03_se2
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_irse.py -x -q --timeout 150 --timeout-method thread > $OUT/pytest_irse.log 2>&1
rc=$?; tail -3 $OUT/pytest_irse.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u tools/loss_trace.py run 20 > $OUT/loss_wall.txt 2>&1
rc=$?; cat $OUT/loss_wall.txt; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/losstr -o p --output-format csv -- python -u tools/loss_trace.py run 20 > $OUT/loss_prof.log 2>&1
rc=$?; [ $rc -ne 0 ] && { tail -20 $OUT/loss_prof.log; exit $rc; }
echo SE2_DONE
