#!/bin/bash
# r06 interleaved A/B of Python knobs on one box: each variant = a quoted list of MODULE.ATTR=VALUE ("" = defaults)
# usage: bash tools/ab/r06_knob_ab.sh TAG ROUNDS "var1" "var2" ...
OUT=gpurun_out/${1:-r06_ab}; ROUNDS=${2:-2}; shift 2
mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    timeout -k 10 300 python tools/bench_knob.py $v -- --steps 30 --warmup 5 --no-cpu-baseline --no-kernel-timer > $OUT/bench_v${i}_$r.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "variant $i bench rc=$rc"; tail -5 $OUT/bench_v${i}_$r.log; exit $rc; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('v%s [%s] round %s:' % tuple(sys.argv[2:5]), d['value'], d['ms_per_step'], flush=True)" $OUT/bench_v${i}_$r.log "$i" "$v" "$r"
  done
done
