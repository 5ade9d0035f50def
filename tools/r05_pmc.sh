#!/bin/bash
# r05 PMC passes: the Winograd F(2x2) r = 1024 forward / data gradient and the split-bf16 direct
# convs (r = 1024 / 128 conv0 data gradient, r = 1024 conv0 transposed forward): wave-state buckets (WAIT_ANY =
# parked on s_waitcnt / barrier, WAIT_INST_ANY = issue stalls, ACTIVE_INST_ANY), MFMA-busy, VALU / LDS / VMEM
# instruction counts, plus any of the optional counters this rocprofv3 lists.  One pass per counter set.
OUT=gpurun_out/${1:-r05_pmc}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1
OPT=""
for c in SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VMEM_WR; do
  grep -qw "$c" $OUT/counters_list.txt && OPT="$OPT $c"
done
OPT=$(echo $OPT | tr ' ' '\n' | head -7 | tr '\n' ' ')
echo "optional counters: $OPT"
run() {  # tag driver args...
  local tag=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU -d $OUT/$tag.a -o p --output-format csv -- python "$@" > $OUT/$tag.a.log 2>&1 || return 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS -d $OUT/$tag.b -o p --output-format csv -- python "$@" > $OUT/$tag.b.log 2>&1 || return 1
  if [ -n "$OPT" ]; then
    timeout -s KILL 90 rocprofv3 --pmc $OPT GRBM_GUI_ACTIVE -d $OUT/$tag.c -o p --output-format csv -- python "$@" > $OUT/$tag.c.log 2>&1 || return 1
  fi
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $OUT/$tag.t -o p --output-format csv -- python "$@" > $OUT/$tag.t.log 2>&1 || return 1
  python tools/pmc_read.py "$OUT/$tag.a/p_counter_collection.csv" "$OUT/$tag.b/p_counter_collection.csv" "$OUT/$tag.c/p_counter_collection.csv" > $OUT/$tag.txt 2>&1
  echo "== $tag"; cat $OUT/$tag.txt
}
run wino_fwd1024 tools/wino_one.py fwd 1024 && run wino_bwd1024 tools/wino_one.py bwd 1024 && \
run x3_bwd0_1024 tools/gemm_one.py bwd_conv0 1024 && run x3_bwd0_128 tools/gemm_one.py bwd_conv0 128 && \
run x3_fwd0_1024 tools/gemm_one.py fwd_conv0 1024 && run x3_fwd0_128 tools/gemm_one.py fwd_conv0 128
