#!/bin/bash
# Round-3 closing pass in one gpurun call: the GPU parity suite (stops at the first failure), then
# tools/gpu_evidence_r3.sh for every bench workload (rocprof trace + PMC traffic + bench line).
#   tools/gpu_final_r3.sh <outdir-prefix>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=${1:-fin}
mkdir -p gpurun_out/${P}_suite
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${P}_suite/pytest_gpu.log 2>&1
rc=$?
tail -2 gpurun_out/${P}_suite/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|E )" gpurun_out/${P}_suite/pytest_gpu.log | head -30; exit $rc; fi
for w in storm flood a2a splitbrain; do
  bash tools/gpu_evidence_r3.sh ${P}_$w $w || exit 1
done
