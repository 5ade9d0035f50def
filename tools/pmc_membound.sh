#!/bin/bash
# PMC passes over tools/bench_membound.py (the HBM-bound synthesis kernels): SQ instruction mix, HBM read / write
# bytes (separate passes, MI355X_MICROARCH.md's rocprofv3 recipe).  usage: bash tools/pmc_membound.sh OUTDIR
OUT=${1:-gpurun_out/pmc_mem}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {  # tag counters...
  local tag=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $OUT/$tag -o p --output-format csv -- python tools/bench_membound.py \
      --res 1024 512 > $OUT/$tag.log 2>&1 || { echo "pass $tag failed"; exit 1; }
}
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD
run grbm GRBM_GUI_ACTIVE
run fetch FETCH_SIZE
run write WRITE_SIZE
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $OUT/t -o p --output-format csv -- python tools/bench_membound.py \
    --res 1024 512 > $OUT/t.log 2>&1 || { echo "trace failed"; exit 1; }
echo PMC_MEM_DONE
