#!/bin/bash
OUT=gpurun_out/r03_wsp
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_wino_sp.py tests/test_gpu_irse.py -x -v --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert" $OUT/pytest.log | tail -30; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u tools/loss_trace.py run 20 > $OUT/loss_wall.txt 2>&1
rc=$?; cat $OUT/loss_wall.txt; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/losstr -o p --output-format csv -- python -u tools/loss_trace.py run 20 > $OUT/loss_prof.log 2>&1
echo WSP_DONE
