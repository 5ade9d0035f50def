#!/bin/bash
# two-level deterministic dd: parity tests (ops dd / blur / act, find_direction bit-equal steps, mapper training) and
# the memory-bound kernels' timing (tools/bench_membound.py: blur_act_bwd / act_bwd with dd at r = 1024 / 512 / 256)
OUT=gpurun_out/${1:-r04_dd2}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ops.py \
  tests/test_gpu_find_direction.py tests/test_gpu_mapper_train.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python tools/bench_membound.py --res 1024 512 256 > $OUT/membound.txt 2>&1 || exit 1
grep -h "blur_act_bwd \|act_bwd " $OUT/membound.txt
