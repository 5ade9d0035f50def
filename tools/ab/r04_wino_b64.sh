#!/bin/bash
# Winograd F(2x2) patch reads as aligned ds_read_b64 pairs over a padded slab: parity, per-layer timing, LDS bank
# conflict counters (r = 1024 forward) and step A/B against _lib_ab/wold (the stride-2 ds_read_b32 reads)
OUT=gpurun_out/${1:-r04_wino_b64}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_wino.py \
  > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in base wold; do
  if [ $v = base ]; then lib=stylemc_amd/_lib/libstylemc_hip.so; else lib=_lib_ab/$v/libstylemc_hip.so; fi
  SMC_HIP_LIB=$lib timeout -k 10 200 python -u tools/bench_wino.py --reps 10 > $OUT/bench_wino_$v.txt 2>&1 || exit 1
  for k in fwd bwd; do
    SMC_HIP_LIB=$lib timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS \
      -d $OUT/pmc_${v}_$k -o p --output-format csv -- python tools/wino_one.py $k 1024 > $OUT/pmc_${v}_$k.log 2>&1 || exit 1
  done
done
python - $OUT <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
for v in ("base", "wold"):
    for k in ("fwd", "bwd"):
        f = glob.glob(os.path.join(out, f"pmc_{v}_{k}", "**", "*counter_collection.csv"), recursive=True)
        tot = collections.Counter()
        for r in csv.DictReader(open(f[0])):
            if "wino_kernel" in r["Kernel_Name"]:
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
        bc, act = tot["SQ_LDS_BANK_CONFLICT"], tot["SQ_LDS_IDX_ACTIVE"]
        print(f"{v} {k} r=1024: bank conflict {bc:.3g} / LDS active {act:.3g} = {bc / max(act, 1):.3f}; LDS insts "
              f"{tot['SQ_INSTS_LDS']:.3g}, wait-LDS {tot['SQ_WAIT_INST_LDS']:.3g}")
PY
grep -h "r=1024\|r= 1024\|1024" $OUT/bench_wino_base.txt $OUT/bench_wino_wold.txt | head -12
bash tools/r04_x3_ab.sh ${OUT#gpurun_out/}/step 2 _lib_ab/wold
