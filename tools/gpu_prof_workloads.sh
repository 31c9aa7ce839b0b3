#!/bin/bash
# rocprofv3 kernel trace + stats of bench.py per workload, summarised per window.
#   tools/gpu_prof_workloads.sh <outdir-under-gpurun_out> <workload>...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-prof}
shift
mkdir -p $OUT
for w in "$@"; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/$w -o run --output-format csv \
    -- python3 -u bench.py --workload $w --no-cpu-baseline --steps 20 --warmup 10 > $OUT/bench_${w}_under_rocprof.log 2>&1 \
    || { echo PROF_FAIL $w; tail -20 $OUT/bench_${w}_under_rocprof.log; exit 1; }
  python3 tools/trace_summary.py $OUT/$w/run_kernel_trace.csv --last 20 --marker k_window_start > $OUT/${w}_trace_summary.txt 2>&1
  echo "== $w"; head -16 $OUT/${w}_trace_summary.txt
done
