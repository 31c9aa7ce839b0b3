#!/bin/bash
# GPU parity suite + plan descriptors on the HIP library (one gpurun call).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-tests}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -5 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error" $OUT/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 200 python -u tools/run_plans.py > $OUT/plans_hip.log 2>&1 || { echo PLANS_FAIL; tail -20 $OUT/plans_hip.log; exit 1; }
cat $OUT/plans_hip.log
