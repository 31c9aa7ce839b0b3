#!/bin/bash
# TCP-acks storm bench, plain and under rocprofv3 (kernel trace + stats).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-tcpp}
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --tcp --tcp-acks --steps 20 --warmup 15 > $OUT/bench_tcp_acks.log 2>&1 || { echo ACKS_FAIL; tail -30 $OUT/bench_tcp_acks.log; exit 1; }
tail -1 $OUT/bench_tcp_acks.log | cut -c1-700
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 -u bench.py --tcp --tcp-acks --steps 20 --warmup 15 > $OUT/bench_under_rocprof.log 2>&1 || { echo PROF_FAIL; tail -20 $OUT/bench_under_rocprof.log; exit 1; }
python3 tools/trace_summary.py $OUT/prof/run_kernel_trace.csv --last 20 > $OUT/trace_summary.txt 2>&1
cat $OUT/trace_summary.txt | head -40
