#!/bin/bash
# Round-2 GPU check in one call: the parity suite (incl. transport-driven shards and the full-size
# sharded configs), then bench.py's sharded path rehearsed with 2 ranks on the one GPU (gloo transport).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r2t}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread --durations=12 > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -16 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "^(FAILED|E )" $OUT/pytest_gpu.log | head -30; exit $rc; }
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 5 --warmup 5 --no-cpu-baseline > $OUT/bench_n2.log 2>&1 || { echo BENCH2_FAIL; tail -30 $OUT/bench_n2.log; exit 1; }
grep '^{' $OUT/bench_n2.log | cut -c1-600
