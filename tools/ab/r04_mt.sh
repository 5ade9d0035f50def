#!/bin/bash
# multi-tile split-bf16 kernel: parity (ops + synthesis + find_direction tests), per-layer timing and step A/B vs
# _lib_ab/mt1 (one row tile per workgroup)
OUT=gpurun_out/${1:-r04_mt}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py \
  tests/test_gpu_find_direction.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python tools/bench_gemm.py > $OUT/base.txt 2>&1 || exit 1
SMC_HIP_LIB=_lib_ab/mt1/libstylemc_hip.so timeout -k 10 200 python tools/bench_gemm.py > $OUT/mt1.txt 2>&1 || exit 1
paste <(grep "r=" $OUT/mt1.txt | awk '{print $1, $2, $3, $(NF-3)}') <(grep "r=" $OUT/base.txt | awk '{print $(NF-3)}')
bash tools/r04_x3_ab.sh ${OUT#gpurun_out/}/step 2 _lib_ab/mt1
