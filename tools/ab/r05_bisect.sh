#!/bin/bash
# r05: which change broke the 2-rank == 1-rank bit equality (tests/test_gpu_distributed.py)?  The product library and
# variants with one r05 feature switched off each.  Stops on anything but a pass / an assertion failure.
OUT=gpurun_out/${1:-r05_bisect}; mkdir -p $OUT
for v in base nolin nowide nowo1 nofold noblur; do
  lib=stylemc_amd/_lib/libstylemc_hip.so; [ $v = base ] || lib=_lib_ab/$v/libstylemc_hip.so
  SMC_HIP_LIB=$lib timeout -k 10 240 python -u -m pytest tests/test_gpu_distributed.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "pipelined_match_single_rank" > $OUT/dist_$v.log 2>&1
  rc=$?; echo "$v rc=$rc: $(tail -1 $OUT/dist_$v.log) $(grep -o "AssertionError: (.*" $OUT/dist_$v.log | head -1)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
