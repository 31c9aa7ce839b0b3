#!/bin/bash
# TCP-mode GPU tests (the staged-overflow regression last), then the TCP storm benches.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-tcpc}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_tcp.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_tcp.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest_tcp.log; exit 1; }
tail -3 $OUT/pytest_tcp.log
timeout -k 10 300 python -u bench.py --tcp --tcp-acks --steps 20 --warmup 15 > $OUT/bench_tcp_acks.log 2>&1 || { echo ACKS_FAIL; tail -30 $OUT/bench_tcp_acks.log; exit 1; }
tail -1 $OUT/bench_tcp_acks.log
