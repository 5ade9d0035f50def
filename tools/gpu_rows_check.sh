set -o pipefail
OUT=gpurun_out/rows1; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "synthesis or find_direction or generate or modconv or torgb" > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || exit 1
grep -o '"value": [0-9.]*, "unit": "images/s", "n_gpus": 1, "steps": 20, "warmup": 5, "ms_per_step": [0-9.]*' $OUT/bench.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof_bench.log 2>&1 || exit 1
python tools/prof_summary.py $OUT/prof/run_kernel_trace.csv > $OUT/kernel_stats.md
