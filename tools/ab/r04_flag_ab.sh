#!/bin/bash
# interleaved bench.py A/B over command-line variants: r04_flag_ab.sh OUT ROUNDS "name1:flags1" "name2:flags2" ...
OUT=gpurun_out/${1:-r04_flag_ab}; ROUNDS=${2:-2}; shift 2
mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    tag=${v%%:*}; flags=${v#*:}
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $flags > $OUT/${tag}_$r.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$tag rc=$rc"; tail -5 $OUT/${tag}_$r.log; exit $rc; }
    python - $OUT/${tag}_$r.log $tag <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]; parts = {k: (v["ms_per_step"], v["frac"]) for k, v in r["parts"].items()}
print(sys.argv[2], d["value"], d["ms_per_step"], (d.get("parity") or {}).get("dir_cosine"), parts, flush=True)
PY
  done
done
