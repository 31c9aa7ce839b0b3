#!/bin/bash
# End-of-milestone GPU evidence, one gpurun call:
#   tools/gpu_round.sh <outdir-under-gpurun_out>
# parity suite -> rocprofv3 kernel trace + stats of the bench -> FETCH_SIZE / WRITE_SIZE passes ->
# per-launch traffic JSON (copied to profiles/r02/ on the box so the final bench line reports it) ->
# the bench with its CPU baseline.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-round}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 15 > $OUT/bench_under_rocprof.log 2>&1 || { echo PROF_FAIL; tail -20 $OUT/bench_under_rocprof.log; exit 1; }
python3 tools/trace_summary.py $OUT/prof/run_kernel_trace.csv --last 20 --marker k_window_start > $OUT/trace_summary.txt 2>&1
KR="k_tb_bucket|k_emit_bucket|k_shape|k_wheel_scatter|k_wheel_hist_rest|k_extract|k_gen_storm|k_bkt"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KR" -d $OUT/pmc_fetch -o run --output-format csv \
  -- python3 -u bench.py --no-cpu-baseline --steps 5 --warmup 5 > $OUT/pmc_fetch.log 2>&1 || { echo PMC_FETCH_FAIL; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KR" -d $OUT/pmc_write -o run --output-format csv \
  -- python3 -u bench.py --no-cpu-baseline --steps 5 --warmup 5 > $OUT/pmc_write.log 2>&1 || { echo PMC_WRITE_FAIL; exit 1; }
python3 tools/pmc_traffic.py $OUT/pmc_fetch/run_counter_collection.csv $OUT/pmc_write/run_counter_collection.csv $OUT/pmc_traffic.json storm 1
mkdir -p profiles/r02 && cp $OUT/pmc_traffic.json profiles/r02/pmc_traffic.json
timeout -k 10 300 python -u bench.py --steps 20 --warmup 15 > $OUT/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
