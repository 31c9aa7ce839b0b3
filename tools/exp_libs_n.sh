#!/bin/bash
# As exp_libs.sh, at several instance counts: tools/exp_libs_n.sh <outdir> <n1> [n2 ...]
set -o pipefail
shopt -s nullglob
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-expn}
shift
mkdir -p $OUT
for n in "$@"; do
for lib in "" tools/exp/*.so; do
  name=$(basename "${lib:-base}" .so)
  TGSIM_LIB=$lib timeout -k 10 120 python -u bench.py --no-cpu-baseline --instances $n --steps 20 --warmup 10 > $OUT/${name}_$n.log 2>&1 || { echo "$name FAIL"; tail -5 $OUT/${name}_$n.log; exit 1; }
  grep '^{' $OUT/${name}_$n.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('%-8s n=%-7s ms/step %.4f  ' % ('$name', '$n', d['ms_per_step']) + ' '.join('%s=%.1f' % (k, v['avg_us']) for k, v in sorted(d['kernels_probe'].items())))"
done
done
