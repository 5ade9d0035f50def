#!/bin/bash
# row-owned attention backward (no memset / atomics) for the 50-token ViT: parity, kernel time, step A/B vs
# _lib_ab/arow0 (the two-query-block form with atomics)
OUT=gpurun_out/${1:-r04_attn}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_vit.py \
  tests/test_gpu_find_direction.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in base arow0; do
  if [ $v = base ]; then lib=stylemc_amd/_lib/libstylemc_hip.so; else lib=_lib_ab/$v/libstylemc_hip.so; fi
  SMC_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run --output-format csv -- \
    python tools/bench_vit.py 4 > $OUT/prof_$v.log 2>&1 || exit 1
  python - $OUT/prof_$v/run_kernel_trace.csv $v <<'PY'
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    for k in ("attn_bwd", "fillBuffer"):
        if k in n:
            d[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in d.items():
    print(sys.argv[2], k, "n", len(v), "avg us", round(sum(v) / len(v), 2))
PY
done
bash tools/r04_x3_ab.sh ${OUT#gpurun_out/}/step 2 _lib_ab/arow0
