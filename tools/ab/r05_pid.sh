#!/bin/bash
# r05: the original image's IR-SE50 features prefetched (on) or computed beside the edited ones in one batch of 8
# (off): run-to-run determinism of each (tools/det_check.py) and interleaved bench rounds.
OUT=gpurun_out/${1:-r05_pid}; mkdir -p $OUT
timeout -k 10 600 python tools/det_check.py pipelined_no_id_prefetch,pipelined 10 > $OUT/det.txt 2>&1 || { echo "det failed"; tail -3 $OUT/det.txt; exit 1; }
grep -v amdgpu $OUT/det.txt
for r in 1 2 3; do for v in on off; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --prefetch-id $v > $OUT/bench_${v}_$r.log 2>&1 || { echo "bench $v failed"; exit 1; }
  echo "$v $(grep -o '"value": [0-9.]*' $OUT/bench_${v}_$r.log)"
done; done
