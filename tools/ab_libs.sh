#!/bin/bash
# Interleaved A/B of library builds (stylemc_amd/build.py with SMC_AB_OUT / SMC_AB_DEFINES) on one box.
# usage: bash tools/ab_libs.sh OUTDIR ROUNDS "VARIANT_DIR ..." -- command args...
# The base library is stylemc_amd/_lib; each variant directory holds a libstylemc_hip.so.  Every step has a limit.
OUT=$1; ROUNDS=$2; VARS=$3; shift 4
mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for v in base $VARS; do
    if [ "$v" = "base" ]; then lib=stylemc_amd/_lib/libstylemc_hip.so; else lib=$v/libstylemc_hip.so; fi
    tag=$(basename $v)
    SMC_HIP_LIB=$lib timeout -k 10 300 "$@" > $OUT/${tag}_$r.txt 2>&1
    rc=$?; echo "[$tag round $r rc=$rc] $(grep -v amdgpu.ids $OUT/${tag}_$r.txt | tail -1 | cut -c1-300)"
    [ $rc -eq 0 ] || exit $rc
  done
done
