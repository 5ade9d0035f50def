#!/bin/bash
# find_direction parity tests, then a step A/B (variants below), fresh processes.
OUT=gpurun_out/r03_graph
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_find_direction.py tests/test_gpu_reference_pins.py tests/test_gpu_mapper_train.py tests/test_gpu_nada.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/sensitivity.py --variants default,unfused --rounds 3 --steps 30 > $OUT/sens.txt 2>&1
rc=$?; cat $OUT/sens.txt | grep -v amdgpu.ids; exit $rc
