#!/bin/bash
# r05 A/B: correctness of each library variant on the direct-conv tests, per-layer conv0 timings
# (tools/bench_gemm.py), then interleaved bench rounds.  usage: bash tools/r05_ab.sh TAG ROUNDS "lib1 lib2 ..."
OUT=gpurun_out/${1:-r05_ab}; ROUNDS=${2:-2}; VARS=${3:-"_lib_ab/wo1"}
mkdir -p $OUT
libof() { if [ "$1" = "base" ]; then echo stylemc_amd/_lib/libstylemc_hip.so; else echo $1/libstylemc_hip.so; fi; }
LIBVARS=$(for v in $VARS; do case $v in tree:*) ;; *) echo $v;; esac; done)
for v in base $LIBVARS; do
  tag=$(basename $v)
  SMC_HIP_LIB=$(libof $v) timeout -k 10 300 python -u -m pytest ${TESTF:-tests/test_gpu_ops.py} -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "${TESTK:-conv_gemm or synthesis_1024 or synthesis_layer}" > $OUT/pytest_$tag.log 2>&1
  rc=$?; echo "$tag tests rc=$rc: $(tail -1 $OUT/pytest_$tag.log)"; [ $rc -eq 0 ] || exit 1
done
for v in base $LIBVARS; do
  tag=$(basename $v)
  SMC_HIP_LIB=$(libof $v) timeout -k 10 200 python ${LAYERTOOL:-tools/bench_gemm.py --only ${ONLY:-fwd_conv0,bwd_conv0}} > $OUT/gemm_$tag.txt 2>&1 || { echo "$tag per-layer tool failed"; tail -3 $OUT/gemm_$tag.txt; exit 1; }
done
python - $OUT base $LIBVARS <<'PY'
import sys, os, re
out = sys.argv[1]; tags = [os.path.basename(v) for v in sys.argv[2:]]
tabs = {}
for t in tags:
    rows = {}
    for l in open(os.path.join(out, f"gemm_{t}.txt")):
        m = re.match(r"(\w+)\s+r=\s*(\d+).*?([\d.]+) us", l)
        if m: rows[(m.group(1), int(m.group(2)))] = float(m.group(3))
    tabs[t] = rows
print("layer".ljust(18) + "".join(t.rjust(10) for t in tags))
for k in tabs[tags[0]]:
    print(f"{k[0]}:{k[1]}".ljust(18) + "".join(f"{tabs[t].get(k, float('nan')):10.1f}" for t in tags))
for t in tags: print(t, "total us", round(sum(tabs[t].values()), 1))
PY
for r in $(seq 1 $ROUNDS); do
  for v in base $VARS; do
    tag=$(basename ${v#tree:})
    case $v in
      tree:*) (cd ${v#tree:} && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline) > $OUT/bench_${tag}_$r.log 2>&1 ;;
      *) SMC_HIP_LIB=$(libof $v) timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_${tag}_$r.log 2>&1 ;;
    esac
    rc=$?; [ $rc -eq 0 ] || { echo "$tag bench rc=$rc"; tail -5 $OUT/bench_${tag}_$r.log; exit $rc; }
    python - $OUT/bench_${tag}_$r.log $tag <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
parts = {k: (v["ms_per_step"], v["frac"]) for k, v in d["roofline"]["parts"].items()}
print(sys.argv[2], d["value"], d["ms_per_step"], parts, flush=True)
PY
  done
done
