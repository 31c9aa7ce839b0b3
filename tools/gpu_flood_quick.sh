#!/bin/bash
# Flood iteration: the flood parity tests (not the full-size one), the quick parity suite, then a
# short flood bench and its rocprofv3 trace summary.   tools/gpu_flood_quick.sh <outdir>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-fquick}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_flood.py tests/test_gpu_parity.py -m gpu -k "not full_size" -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -2 $OUT/pytest.log
[ $rc -ne 0 ] && { grep -E "^(FAILED|E )" $OUT/pytest.log | head -30; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 -u bench.py --workload flood --no-cpu-baseline --steps 20 --warmup 100 > $OUT/bench_under_rocprof.log 2>&1 || { echo PROF_FAIL; tail -20 $OUT/bench_under_rocprof.log; exit 1; }
python3 tools/trace_summary.py $OUT/prof/run_kernel_trace.csv --last 20 --marker k_window_start > $OUT/trace_summary.txt 2>&1
head -25 $OUT/trace_summary.txt
timeout -k 10 300 python -u bench.py --workload flood --no-cpu-baseline > $OUT/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-400
