#!/bin/bash
# GPU parity suite (stops at the first failure), then one short bench line per named workload.
#   tools/gpu_suite_bench.sh <outdir-under-gpurun_out> <workload>...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-sb}
shift
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E )" $OUT/pytest_gpu.log | head -30; exit $rc; fi
for w in "$@"; do
  case $w in flood) WARM=100;; *) WARM=10;; esac
  timeout -k 10 200 python -u bench.py --workload $w --no-cpu-baseline --steps 30 --warmup $WARM > $OUT/bench_$w.log 2>&1 || { echo BENCH_FAIL $w; tail -20 $OUT/bench_$w.log; exit 1; }
  grep '^{' $OUT/bench_$w.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('$w value %.4e ms/step %.4f ' % (d['value'], d['ms_per_step']) + ' '.join('%s=%.1f' % (k, v['avg_us']) for k, v in sorted(d.get('kernels_probe', {}).items())))"
done
