#!/bin/bash
# Round-3 first GPU pass: the whole gpu suite, then one bench line per workload (storm / flood / a2a /
# splitbrain) and a rocprofv3 kernel trace of the storm bench. Stops at the first failing step.
#   tools/gpu_r3_first.sh <outdir-under-gpurun_out>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3first}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for w in storm flood a2a splitbrain; do
  timeout -k 10 200 python -u bench.py --workload $w --steps 20 --warmup 10 > $OUT/bench_$w.log 2>&1 || { echo BENCH_FAIL $w; tail -30 $OUT/bench_$w.log; exit 1; }
  tail -1 $OUT/bench_$w.log | cut -c1-400
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 15 > $OUT/bench_under_rocprof.log 2>&1 || { echo PROF_FAIL; tail -20 $OUT/bench_under_rocprof.log; exit 1; }
python3 tools/trace_summary.py $OUT/prof/run_kernel_trace.csv --last 20 --marker k_window_start > $OUT/trace_summary.txt 2>&1
head -30 $OUT/trace_summary.txt
