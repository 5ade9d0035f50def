#!/bin/bash
# r05: one-batch attention staging (base) vs the r05 HEAD attention kernels (oldattn, same split planning): rocprof
# kernel stats of tools/bench_vit.py 8 under each library, then the full GPU suite on the base library.
OUT=gpurun_out/${1:-r05_attn}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base oldattn; do
  lib=stylemc_amd/_lib/libstylemc_hip.so; [ $v = base ] || lib=_lib_ab/$v/libstylemc_hip.so
  SMC_HIP_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o p --output-format csv -- python tools/bench_vit.py 8 > $OUT/vit8_$v.txt 2>&1 || { echo "prof $v failed"; tail -5 $OUT/vit8_$v.txt; exit 1; }
  echo "== $v"; grep hip $OUT/vit8_$v.txt; find $OUT/prof_$v -name "*kernel_stats.csv" -exec grep -h "attn_" {} \; | cut -c1-200
done
bash tools/gpu_tests.sh r05_attn "tests/test_gpu_ops.py tests/test_gpu_wino.py tests/test_gpu_vit.py" full
