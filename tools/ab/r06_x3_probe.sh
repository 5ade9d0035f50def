# split-bf16 F(2x2) (wino_x3_kernel) at r = 1024: tests, then the synthesis-epilogue timings of the product library,
# the fp32 kernel (--no-split: no workspace) and variant libraries under ab_r06/ (SMC_HIP_LIB)
mkdir -p gpurun_out/x3f
set -o pipefail
true
timeout -k 10 100 python tools/bench_wino.py --res 1024 --modact --no-split > gpurun_out/x3f/fp32.log 2>&1 || exit 1
timeout -k 10 100 python tools/bench_wino.py --res 1024 --modact > gpurun_out/x3f/prod.log 2>&1 || exit 1
for v in $(ls ab_r06); do SMC_HIP_LIB=ab_r06/$v/libstylemc_hip.so timeout -k 10 100 python tools/bench_wino.py --res 1024 --modact > gpurun_out/x3f/$v.log 2>&1 || exit 1; done
timeout -k 10 100 python tools/bench_wino.py --res 1024 --modact > gpurun_out/x3f/prod2.log 2>&1 || exit 1
