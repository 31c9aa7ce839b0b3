#!/bin/bash
# TCP GPU tests, then the TCP-acks storm under rocprofv3 (kernel trace summary).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-tcpi}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_tcp.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_tcp.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest_tcp.log; exit 1; }
tail -1 $OUT/pytest_tcp.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 -u bench.py --tcp --tcp-acks --steps 20 --warmup 15 > $OUT/bench_under_rocprof.log 2>&1 || { echo PROF_FAIL; tail -20 $OUT/bench_under_rocprof.log; exit 1; }
grep '^{' $OUT/bench_under_rocprof.log | cut -c1-300
python3 tools/trace_summary.py $OUT/prof/run_kernel_trace.csv --last 20 > $OUT/trace_summary.txt 2>&1
head -16 $OUT/trace_summary.txt
