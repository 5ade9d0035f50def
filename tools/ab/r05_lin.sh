#!/bin/bash
# r05: ViT GEMM K sweep (tools/lin_sweep.py, cold weights) and the tower (tools/bench_vit.py) for the ring / K-split
# variants of lin_gemm2_kernel: base (NST 2, KW 2), n2k1, n3k1, n4k1.
OUT=gpurun_out/${1:-r05_lin}
mkdir -p $OUT
for v in base n2k1 n3k1 n4k1; do
  lib=stylemc_amd/_lib/libstylemc_hip.so; [ $v = base ] || lib=_lib_ab/$v/libstylemc_hip.so
  SMC_HIP_LIB=$lib timeout -k 10 200 python tools/lin_sweep.py > $OUT/sweep_$v.txt 2>&1 || { echo "sweep $v failed"; tail -5 $OUT/sweep_$v.txt; exit 1; }
  SMC_HIP_LIB=$lib timeout -k 10 200 python tools/bench_vit.py 4 > $OUT/vit4_$v.txt 2>&1 || { echo "vit $v failed"; tail -5 $OUT/vit4_$v.txt; exit 1; }
  SMC_HIP_LIB=$lib timeout -k 10 200 python tools/bench_vit.py 8 > $OUT/vit8_$v.txt 2>&1 || { echo "vit8 $v failed"; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $OUT/sweep_$v.txt; grep hip $OUT/vit4_$v.txt $OUT/vit8_$v.txt
done
