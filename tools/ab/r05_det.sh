#!/bin/bash
# r05: run-to-run determinism of the pipelined step (tools/det_check.py) with the ViT GEMMs' in-launch split-K
# hand-off as it is (base), with sc1 partial-tile loads (sc1ld), and replaced by the reduction kernel (noinl); then
# interleaved bench rounds of the three.
OUT=gpurun_out/${1:-r05_det}; mkdir -p $OUT
for v in base noinl sc1ld; do
  lib=stylemc_amd/_lib/libstylemc_hip.so; [ $v = base ] || lib=_lib_ab/$v/libstylemc_hip.so
  SMC_HIP_LIB=$lib timeout -k 10 400 python tools/det_check.py pipelined 6 > $OUT/det_$v.txt 2>&1 || { echo "det $v failed"; tail -3 $OUT/det_$v.txt; exit 1; }
  echo "$v: $(grep -v amdgpu $OUT/det_$v.txt)"
done
for r in 1 2; do for v in base noinl sc1ld; do
  lib=stylemc_amd/_lib/libstylemc_hip.so; [ $v = base ] || lib=_lib_ab/$v/libstylemc_hip.so
  SMC_HIP_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_${v}_$r.log 2>&1 || { echo "bench $v failed"; exit 1; }
  echo "$v $(grep -o '"value": [0-9.]*' $OUT/bench_${v}_$r.log)"
done; done
