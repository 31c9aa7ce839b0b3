#!/bin/bash
# One iteration on the GPU box: parity suite, then a short bench (no CPU baseline).
#   tools/gpu_iter.sh <outdir> [bench args...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-iter}
shift
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E )" $OUT/pytest_gpu.log | head -30; exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --warmup 20 "$@" > $OUT/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('value %.3e msgs/s  ms/step %.3f  dominant %s frac %.3f' % (d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac']))
for k,v in sorted(d['kernels_probe'].items(), key=lambda kv: -kv[1]['avg_us']*kv[1]['launches']):
    print('  %-16s %8.2f us x %d' % (k, v['avg_us'], v['launches']))
"
