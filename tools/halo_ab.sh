# A/B of the opt-in halo-tile conv kernel (conv3_halo_kernel, SMC_HALO=1) against the default tap-major LDS-DMA
# GEMM: parity of both paths on the 32-channel shapes, then per-layer timings (tools/bench_gemm.py).
#   usage: bash tools/halo_ab.sh TAG        (extra knobs for the halo path: SMC_HALO_CK=4, SMC_HALO_TM=2)
set -o pipefail
OUT=gpurun_out/${1:-halo}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "32ch or synthesis_layer or synthesis_1024" > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; grep -E "^E  " $OUT/pytest.log | head; [ $rc -eq 0 ] || exit $rc
SMC_HALO=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "32ch or synthesis_1024" > $OUT/pytest_halo.log 2>&1; rc=$?; tail -2 $OUT/pytest_halo.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_gemm.py > $OUT/gemm_default.log 2>&1 || exit 1
SMC_HALO=1 timeout -k 10 200 python tools/bench_gemm.py > $OUT/gemm_halo.log 2>&1 || exit 1
grep -E "conv1  r= 1024|TOTAL" $OUT/gemm_default.log $OUT/gemm_halo.log
