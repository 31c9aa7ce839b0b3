#!/bin/bash
# Round-3 GPU pass that reports every failing test (no -x), then - unless the suite crashed the
# process (abort / segfault / time limit) - one bench line per workload.
#   tools/gpu_r3_all.sh <outdir-under-gpurun_out> [pytest selection...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3all}
shift
mkdir -p $OUT
SEL=${@:-tests}
timeout -k 10 900 python -u -m pytest $SEL -m gpu -v --timeout 240 --timeout-method thread --durations=15 -rf > $OUT/pytest_gpu.log 2>&1
rc=$?
grep -E "^(FAILED|ERROR)|passed|failed" $OUT/pytest_gpu.log | tail -40
case $rc in 0|1) ;; *) echo "PYTEST rc=$rc: stopping"; exit $rc;; esac
if [ -n "$NOBENCH" ]; then exit $rc; fi
for w in storm flood a2a splitbrain; do
  timeout -k 10 200 python -u bench.py --workload $w --steps 20 --warmup 10 > $OUT/bench_$w.log 2>&1 || { echo BENCH_FAIL $w; tail -30 $OUT/bench_$w.log; exit 1; }
  tail -1 $OUT/bench_$w.log | cut -c1-600
done
exit $rc
