#!/bin/bash
# GEMM layer-set timing (tools/bench_gemm.py) after the op tests.  usage: bash tools/gemm_ab.sh TAG [pytest -k]
TAG=${1:-gemm}; K=${2:-"conv_gemm or synthesis"}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread -k "$K" > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log; case $rc in 0) ;; 1) exit 1;; *) echo "pytest rc=$rc"; exit $rc;; esac
timeout -k 10 300 python tools/bench_gemm.py --reps 10 > $OUT/bench_gemm.txt 2>&1; rc=$?
cat $OUT/bench_gemm.txt; exit $rc
