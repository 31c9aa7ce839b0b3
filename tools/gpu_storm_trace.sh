#!/bin/bash
# Storm (headline) per-window kernel trace: rocprofv3 trace + stats of a short bench run and the
# per-window summary.   tools/gpu_storm_trace.sh <outdir> [extra bench args]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-strace}
shift
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 "$@" > $OUT/bench_under_rocprof.log 2>&1 || { echo PROF_FAIL; tail -20 $OUT/bench_under_rocprof.log; exit 1; }
python3 tools/trace_summary.py $OUT/prof/run_kernel_trace.csv --last 20 --marker k_window_start > $OUT/trace_summary.txt 2>&1
head -30 $OUT/trace_summary.txt
