set -o pipefail
OUT=gpurun_out/convt_ab; mkdir -p $OUT
timeout -k 10 200 python tools/bench_gemm.py --reps 20 > $OUT/default.log 2>&1 || exit 1
SMC_NO_CONVT_FUSION=1 timeout -k 10 200 python tools/bench_gemm.py --reps 20 > $OUT/nofuse.log 2>&1 || exit 1
SMC_CONVT_BM=256 timeout -k 10 200 python tools/bench_gemm.py --reps 20 > $OUT/bm256.log 2>&1 || exit 1
grep -E "fwd_conv0  r= (512|1024)|TOTAL" $OUT/default.log $OUT/nofuse.log $OUT/bm256.log
