#!/bin/bash
# Quick iteration: parity suite without the full-size tests, then the experiment libraries' timing.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-quick}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_correlation.py tests/test_topics.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -2 $OUT/pytest.log
[ $rc -ne 0 ] && { grep -E "^(FAILED|E )" $OUT/pytest.log | head -30; exit $rc; }
bash tools/exp_libs.sh ${1:-quick}
