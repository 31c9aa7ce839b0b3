#!/bin/bash
# TCP-mode storm benches (no ACKs, then ACKs on the reverse path), one gpurun call.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-tcpb}
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --tcp --steps 20 --warmup 15 > $OUT/bench_tcp.log 2>&1 || { echo TCP_FAIL; tail -30 $OUT/bench_tcp.log; exit 1; }
tail -1 $OUT/bench_tcp.log | cut -c1-400
timeout -k 10 300 python -u bench.py --tcp --tcp-acks --steps 20 --warmup 15 > $OUT/bench_tcp_acks.log 2>&1 || { echo ACKS_FAIL; tail -30 $OUT/bench_tcp_acks.log; exit 1; }
tail -1 $OUT/bench_tcp_acks.log
