#!/bin/bash
# Round-3 evidence for one workload, one gpurun call: rocprofv3 kernel trace + stats of the bench,
# FETCH_SIZE / WRITE_SIZE passes (one counter per run, MI355X_MICROARCH.md HBM section) -> a
# hash-stamped profiles/r03/pmc_traffic[_<w>].json on the box (bench.py reports it as traffic), then
# the bench line itself with its CPU baseline.
#   tools/gpu_evidence_r3.sh <outdir-under-gpurun_out> <storm|flood|a2a|splitbrain> [bench args...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-ev}
W=${2:-storm}
shift 2
mkdir -p $OUT profiles/r03
case $W in
  storm) WARM="--warmup 15"; SUF="";;
  flood) WARM="--warmup 100"; SUF="_flood";;
  *) WARM="--warmup 10"; SUF="_$W";;
esac
B="bench.py --workload $W --no-cpu-baseline $WARM $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$W -o run --output-format csv \
  -- python3 -u $B --steps 20 > $OUT/bench_${W}_under_rocprof.log 2>&1 || { echo PROF_FAIL; tail -20 $OUT/bench_${W}_under_rocprof.log; exit 1; }
python3 tools/trace_summary.py $OUT/prof_$W/run_kernel_trace.csv --last 20 --marker k_window_start > $OUT/${W}_trace_summary.txt 2>&1
head -14 $OUT/${W}_trace_summary.txt
KR="k_tb_bucket|k_emit_bucket|k_extract_shape|k_wheel_scatter|k_extract|k_shape|k_gen_storm|k_bkt|k_local_hist|k_flood|k_seg_small|k_rest|k_window_start|k_probe"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $c --kernel-include-regex "$KR" -d $OUT/pmc_${W}_$c -o run --output-format csv \
    -- python3 -u $B --steps 5 > $OUT/pmc_${W}_$c.log 2>&1 || { echo PMC_FAIL $c; tail -5 $OUT/pmc_${W}_$c.log; exit 1; }
done
python3 tools/pmc_traffic.py $OUT/pmc_${W}_FETCH_SIZE/run_counter_collection.csv $OUT/pmc_${W}_WRITE_SIZE/run_counter_collection.csv \
  $OUT/pmc_traffic$SUF.json $W 1
cp $OUT/pmc_traffic$SUF.json profiles/r03/pmc_traffic$SUF.json
timeout -k 10 300 python3 -u bench.py --workload $W $WARM $* > $OUT/bench_$W.log 2>&1 || { echo BENCH_FAIL; tail -30 $OUT/bench_$W.log; exit 1; }
tail -1 $OUT/bench_$W.log | cut -c1-400
