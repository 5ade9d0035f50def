# per-launch A/B of a variant library (SMC_HIP_LIB) against the product on the synthesis conv shapes, interleaved
# usage: bash tools/ab/r06_lib_launch_ab.sh TAG VARIANT_DIR [bench_wino args...]
OUT=gpurun_out/$1; V=$2; shift 2
mkdir -p $OUT
for r in 1 2; do
  timeout -k 10 150 python tools/bench_wino.py "$@" > $OUT/prod_$r.log 2>&1 || exit 1
  SMC_HIP_LIB=$V/libstylemc_hip.so timeout -k 10 150 python tools/bench_wino.py "$@" > $OUT/var_$r.log 2>&1 || exit 1
done
grep -H "r=" $OUT/*.log | sed 's/direct.*wino / wino /'
