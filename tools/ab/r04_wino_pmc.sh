#!/bin/bash
# Where the F(2x2) kernel's LDS bank-conflict cycles come from: counters on the r = 1024 forward for the library,
# PROBE 3 (no U / patch DMAs after the first K step) and PROBE 32 (no LDS fragment reads)
OUT=gpurun_out/${1:-r04_wino_pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base wp3 wp32; do
  if [ $v = base ]; then lib=stylemc_amd/_lib/libstylemc_hip.so; else lib=_lib_ab/$v/libstylemc_hip.so; fi
  SMC_HIP_LIB=$lib timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS \
    -d $OUT/pmc_$v -o p --output-format csv -- python tools/wino_one.py fwd 1024 > $OUT/pmc_$v.log 2>&1 || exit 1
done
python - $OUT <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
for v in ("base", "wp3", "wp32"):
    f = glob.glob(os.path.join(out, f"pmc_{v}", "**", "*counter_collection.csv"), recursive=True)
    tot = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        if "wino_kernel" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
    bc, act = tot["SQ_LDS_BANK_CONFLICT"], tot["SQ_LDS_IDX_ACTIVE"]
    print(f"{v}: bank conflict {bc:.4g} / LDS active {act:.4g} = {bc / max(act, 1):.3f}; LDS insts {tot['SQ_INSTS_LDS']:.4g}")
PY
