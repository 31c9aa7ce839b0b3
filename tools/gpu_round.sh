set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r1/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/r1/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r1/pytest_gpu.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 15 > gpurun_out/r1/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/r1/bench.log; exit 1; }
tail -1 gpurun_out/r1/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r1/prof -o run --output-format csv -- python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 15 > gpurun_out/r1/prof_bench.log 2>&1 || { echo PROF_FAIL; tail -30 gpurun_out/r1/prof_bench.log; exit 1; }
tail -1 gpurun_out/r1/prof_bench.log
