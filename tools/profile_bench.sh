#!/bin/bash
# rocprofv3 kernel trace + stats of the bench command (the summary the bench roofline must agree with).
#   tools/profile_bench.sh <outdir-under-gpurun_out> [bench args...]
set -o pipefail
OUT=${1:-prof}
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$OUT -o run --output-format csv \
  -- python3 -u bench.py --no-cpu-baseline "$@" > gpurun_out/$OUT/bench.log 2>&1
rc=$?
tail -1 gpurun_out/$OUT/bench.log
exit $rc
