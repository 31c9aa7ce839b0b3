#!/bin/bash
# End-of-round evidence in one gpurun call: the storm (parity suite, rocprofv3 trace + stats, PMC
# FETCH/WRITE passes, bench with CPU baseline), the flood (trace, PMC, bench), the TCP benches.
#   tools/gpu_final.sh <outdir-under-gpurun_out>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${1:-final}
bash tools/gpu_round.sh $OUT/storm || exit 1
bash tools/gpu_flood_round.sh $OUT/flood || exit 1
timeout -k 10 300 python -u bench.py --tcp --steps 20 --warmup 15 > gpurun_out/$OUT/bench_tcp.log 2>&1 || { echo TCP_FAIL; exit 1; }
timeout -k 10 300 python -u bench.py --tcp --tcp-acks --steps 20 --warmup 15 > gpurun_out/$OUT/bench_tcp_acks.log 2>&1 || { echo ACKS_FAIL; exit 1; }
grep -h '^{' gpurun_out/$OUT/bench_tcp.log gpurun_out/$OUT/bench_tcp_acks.log | cut -c1-200
