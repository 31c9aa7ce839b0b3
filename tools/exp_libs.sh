#!/bin/bash
# Times the bench's kernel classes with each experiment build in tools/exp/ (TGSIM_LIB) beside the
# in-tree library.   tools/exp_libs.sh <outdir>
set -o pipefail
shopt -s nullglob
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-exp}
mkdir -p $OUT
for lib in "" tools/exp/*.so; do
  name=$(basename "${lib:-base}" .so)
  TGSIM_LIB=$lib timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 20 --warmup 10 > $OUT/$name.log 2>&1 || { echo "$name FAIL"; tail -5 $OUT/$name.log; exit 1; }
  grep '^{' $OUT/$name.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
print('%-14s ms/step %.4f  ' % ('$name', d['ms_per_step']) + ' '.join('%s=%.1f' % (k, v['avg_us']) for k, v in sorted(d['kernels_probe'].items())))"
done
