#!/bin/bash
# LayerNorm forward / backward with the operands loaded before the stores: parity, kernel time, step A/B vs _lib_ab/lnprev
OUT=gpurun_out/${1:-r04_ln}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_vit.py \
  tests/test_gpu_find_direction.py > $OUT/pytest.log 2>&1 \
  || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in base lnprev; do
  if [ $v = base ]; then lib=stylemc_amd/_lib/libstylemc_hip.so; else lib=_lib_ab/$v/libstylemc_hip.so; fi
  SMC_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run --output-format csv -- \
    python bench.py --steps 5 --warmup 2 --no-cpu-baseline --roofline-steps 0 > $OUT/prof_$v.log 2>&1 || exit 1
  python - $OUT/prof_$v/run_kernel_trace.csv $v <<'PY'
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "ln_" in r["Kernel_Name"]:
        d[r["Kernel_Name"].split("(")[1][:40] if False else r["Kernel_Name"][:45]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in d.items():
    print(sys.argv[2], k, "n", len(v), "avg us", round(sum(v) / len(v), 1))
PY
done
bash tools/r04_x3_ab.sh ${OUT#gpurun_out/}/step 2 _lib_ab/lnprev
