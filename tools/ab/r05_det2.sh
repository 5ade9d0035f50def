#!/bin/bash
# r05: the pipelined step after recording the side stream on every tensor it reads from another stream: run-to-run
# determinism (tools/det_check.py, 8 runs), the 2-rank == 1-rank test three times, a bench line.
OUT=gpurun_out/${1:-r05_det2}; mkdir -p $OUT
timeout -k 10 500 python tools/det_check.py pipelined,pipelined_no_id_prefetch 8 > $OUT/det.txt 2>&1 || { echo "det failed"; tail -3 $OUT/det.txt; exit 1; }
grep -v amdgpu $OUT/det.txt
for r in 1 2 3; do
  timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py -m gpu -x -q --timeout 250 --timeout-method thread -p no:cacheprovider > $OUT/dist_$r.log 2>&1
  rc=$?; echo "dist run $r rc=$rc: $(tail -1 $OUT/dist_$r.log)"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.log 2>&1 && grep -o '"value": [0-9.]*' $OUT/bench.log
