#!/bin/bash
# PMC counters for single GEMM shapes. usage: bash tools/pmc_gemm.sh OUTDIR "fwd_conv1 1024" "fwd_conv1 128" ...
OUT=$1; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for spec in "$@"; do
  set -- $spec
  tag=${1}_$2
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU -d $OUT/$tag.a -o p --output-format csv -- python ${ONE:-tools/gemm_one.py} $1 $2 > $OUT/$tag.a.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d $OUT/$tag.b -o p --output-format csv -- python ${ONE:-tools/gemm_one.py} $1 $2 > $OUT/$tag.b.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/$tag.c -o p --output-format csv -- python ${ONE:-tools/gemm_one.py} $1 $2 > $OUT/$tag.c.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/$tag.d -o p --output-format csv -- python ${ONE:-tools/gemm_one.py} $1 $2 > $OUT/$tag.d.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/$tag.t -o p --output-format csv -- python ${ONE:-tools/gemm_one.py} $1 $2 > $OUT/$tag.t.log 2>&1 || exit 1
done
echo PMC_DONE
