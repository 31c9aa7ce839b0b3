#!/bin/bash
# Rehearse the sharded bench on a one-GPU box: N ranks share cuda:0, collectives over gloo.
# The timed deliveries of every N must equal the single-shard run's (same rounds, bit-exact shards).
#   tools/gpu_rehearse.sh <outdir> [N...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-rehearse}
shift
mkdir -p $OUT
ARGS="--no-cpu-baseline --steps 8 --warmup 4"
timeout -k 10 200 python -u bench.py --gpus 1 $ARGS > $OUT/bench_n1.log 2>&1 || { echo N1_FAIL; tail -20 $OUT/bench_n1.log; exit 1; }
for n in "${@:-2}"; do
  timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29500 + n)) bench.py --gpus $n $ARGS > $OUT/bench_n$n.log 2>&1 \
    || { echo N${n}_FAIL; tail -30 $OUT/bench_n$n.log; exit 1; }
done
for f in $OUT/bench_n*.log; do
  grep '^{' $f | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('%s value %.3e ms/step %.3f delivered %d' % ('$f', d['value'], d['ms_per_step'], d['config']['delivered_in_timed_steps']))"
done
