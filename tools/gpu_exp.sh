set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/exp1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/exp1/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/exp1/pytest.log
[ $rc -ne 0 ] && { grep -E "^(FAILED|E )" gpurun_out/exp1/pytest.log | head -20; exit 1; }
bash tools/exp_libs.sh exp1
