#!/bin/bash
# Graph-captured prefetch: the find_direction parity tests, then step A/B (graph vs eager prefetch), fresh processes.
OUT=gpurun_out/r03_graph
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_find_direction.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/sensitivity.py --variants default,graph --rounds 3 --steps 30 > $OUT/sens.txt 2>&1
rc=$?; cat $OUT/sens.txt | grep -v amdgpu.ids; exit $rc
