#!/bin/bash
# Round-3 GPU check: the given pytest selection (default: the whole gpu suite), one call.
#   tools/gpu_r3.sh <outdir-under-gpurun_out> [pytest args...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3}
shift
mkdir -p $OUT
ARGS=${@:-tests}
timeout -k 10 1000 python -u -m pytest $ARGS -m gpu -x -v --timeout 900 --timeout-method thread --durations=20 > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -25 $OUT/pytest_gpu.log
exit $rc
