#!/bin/bash
# The storm on a 12.5k-instance shard (the per-GPU share at 8 GPUs): bench + rocprofv3 trace summary.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-small}
mkdir -p $OUT
timeout -k 10 200 python -u bench.py --instances 12500 --no-cpu-baseline --steps 50 --warmup 20 > $OUT/bench_12k.log 2>&1 || { echo B_FAIL; tail -20 $OUT/bench_12k.log; exit 1; }
grep '^{' $OUT/bench_12k.log | cut -c1-420
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 -u bench.py --instances 12500 --no-cpu-baseline --steps 50 --warmup 20 > $OUT/bench_under_rocprof.log 2>&1 || { echo PROF_FAIL; tail -20 $OUT/bench_under_rocprof.log; exit 1; }
python3 tools/trace_summary.py $OUT/prof/run_kernel_trace.csv --last 50 > $OUT/trace_summary.txt 2>&1
head -16 $OUT/trace_summary.txt
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 30 --warmup 20 > $OUT/bench_100k.log 2>&1 || { echo B2_FAIL; tail -20 $OUT/bench_100k.log; exit 1; }
grep '^{' $OUT/bench_100k.log | cut -c1-300
