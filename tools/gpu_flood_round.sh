#!/bin/bash
# Config 5 evidence in one gpurun call: rocprofv3 trace + stats of the flood bench, FETCH_SIZE /
# WRITE_SIZE passes (-> profiles/r02/pmc_traffic_flood.json on the box), the bench line with its
# CPU baseline.   tools/gpu_flood_round.sh <outdir-under-gpurun_out>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-flood}
mkdir -p $OUT
B="bench.py --workload flood --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv \
  -- python3 -u $B --steps 20 --warmup 100 > $OUT/bench_under_rocprof.log 2>&1 || { echo PROF_FAIL; tail -20 $OUT/bench_under_rocprof.log; exit 1; }
python3 tools/trace_summary.py $OUT/prof/run_kernel_trace.csv --last 20 --marker k_window_start > $OUT/trace_summary.txt 2>&1
KR="k_tb_bucket|k_emit_bucket|k_extract_shape|k_wheel_scatter|k_extract|k_flood|k_bkt|k_local_hist"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KR" -d $OUT/pmc_fetch -o run --output-format csv \
  -- python3 -u $B --steps 5 --warmup 100 > $OUT/pmc_fetch.log 2>&1 || { echo PMC_FETCH_FAIL; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KR" -d $OUT/pmc_write -o run --output-format csv \
  -- python3 -u $B --steps 5 --warmup 100 > $OUT/pmc_write.log 2>&1 || { echo PMC_WRITE_FAIL; exit 1; }
python3 tools/pmc_traffic.py $OUT/pmc_fetch/run_counter_collection.csv $OUT/pmc_write/run_counter_collection.csv $OUT/pmc_traffic_flood.json flood 1
mkdir -p profiles/r02 && cp $OUT/pmc_traffic_flood.json profiles/r02/pmc_traffic_flood.json
timeout -k 10 300 python -u bench.py --workload flood > $OUT/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-300
