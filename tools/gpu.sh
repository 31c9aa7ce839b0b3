#!/bin/bash
# One parameterised GPU-box entry point (run under gpurun; every GPU step has its own time limit and
# the steps are chained so a failure ends the call):
#   tools/gpu.sh tests <out> [pytest args...]         pytest -m gpu (default: the whole GPU suite)
#   tools/gpu.sh bench <out> <workload> [bench args]   one bench line
#   tools/gpu.sh evidence <out> <workload> <round> [bench args]
#        rocprofv3 kernel trace + stats of the bench (<w>_kernel_stats.csv, <w>_trace_summary.txt),
#        FETCH_SIZE / WRITE_SIZE passes over every tgsim kernel (one counter per run, the guide's HBM
#        section) -> hash-stamped
#        pmc_traffic[_<w>].json, then the bench line (bench_<w>.json) - all into
#        gpurun_out/<out>/profiles/<round>/ (only gpurun_out/ comes back from the box: copy that
#        directory into profiles/<round>/ here)
#   tools/gpu.sh pmc <out> <workload> [bench args]     SQ / LDS / TCC / HBM counter groups, one run each
#   tools/gpu.sh ab <out> <rounds> <workload> <name>... interleaved timing of libtgsim_<name>.so builds
#        (tools/build_variant.sh) against the product library
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MODE=$1; OUT=gpurun_out/$2; shift 2
mkdir -p $OUT
warm() { case $1 in storm) echo "--warmup 15";; flood) echo "--warmup 100";; *) echo "--warmup 10";; esac; }
suffix() { [ "$1" = storm ] && echo "" || echo "_$1"; }
KR="k_tb_bucket|k_emit_bucket|k_extract_shape|k_wheel_scatter|k_extract|k_shape|k_gen_storm|k_bkt|k_local_hist|k_flood|k_seg_small|k_rest|k_window_start|k_probe|k_storm"
case $MODE in
tests)
  [ $# -eq 0 ] && set -- tests
  timeout -k 10 1000 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu "$@" > $OUT/tests.log 2>&1
  rc=$?; grep -E "passed|failed|error" $OUT/tests.log | tail -3; [ $rc -eq 0 ] || tail -40 $OUT/tests.log; exit $rc;;
bench)
  W=$1; shift
  timeout -k 10 400 python3 -u bench.py --workload $W $(warm $W) "$@" > $OUT/bench_$W.log 2>&1 || { echo BENCH_FAIL; tail -30 $OUT/bench_$W.log; exit 1; }
  tail -1 $OUT/bench_$W.log | cut -c1-600;;
evidence)
  W=$1; R=$2; shift 2
  P=$OUT/profiles/$R
  mkdir -p $P
  # the profiled runs leave out the storm line's flood beside it (its windows would mix into the
  # storm's trace and counters); the bench line at the end keeps it
  NB=""; [ "$W" = storm ] && NB="--no-beside"
  B="bench.py --workload $W --no-cpu-baseline $NB $(warm $W) $*"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$W -o run --output-format csv \
    -- python3 -u $B --steps 20 > $OUT/bench_${W}_under_rocprof.log 2>&1 || { echo PROF_FAIL; tail -20 $OUT/bench_${W}_under_rocprof.log; exit 1; }
  cp $OUT/prof_$W/run_kernel_stats.csv $P/${W}_kernel_stats.csv
  python3 tools/trace_summary.py $OUT/prof_$W/run_kernel_trace.csv --last 20 --marker k_window_start > $P/${W}_trace_summary.txt 2>&1
  head -16 $P/${W}_trace_summary.txt
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $c --kernel-include-regex "k_" -d $OUT/pmc_${W}_$c -o run --output-format csv \
      -- python3 -u $B --steps 5 > $OUT/pmc_${W}_$c.log 2>&1 || { echo PMC_FAIL $c; tail -5 $OUT/pmc_${W}_$c.log; exit 1; }
  done
  # the flood publishes every 4 windows: its per-window sums average two whole cycles
  LAST=5; [ "$W" = flood ] && LAST=8
  python3 tools/pmc_traffic.py $OUT/pmc_${W}_FETCH_SIZE/run_counter_collection.csv $OUT/pmc_${W}_WRITE_SIZE/run_counter_collection.csv \
    $P/pmc_traffic$(suffix $W).json $W 1 --last $LAST || exit 1
  timeout -k 10 400 python3 -u bench.py --workload $W $(warm $W) "$@" > $OUT/bench_$W.log 2>&1 || { echo BENCH_FAIL; tail -30 $OUT/bench_$W.log; exit 1; }
  tail -1 $OUT/bench_$W.log > $P/bench_$W.json
  cut -c1-600 $P/bench_$W.json;;
pmc)
  W=$1; shift
  B="bench.py --workload $W --no-cpu-baseline --steps 5 $(warm $W) $*"
  run() {
    timeout -s KILL 150 rocprofv3 --pmc $2 --kernel-include-regex "$KR" -d $OUT/$1 -o run --output-format csv \
      -- python3 -u $B > $OUT/$1.log 2>&1 || { echo "PMC_FAIL $1"; tail -5 $OUT/$1.log; exit 1; }
    python3 tools/pmc_table.py $OUT/$1/run_counter_collection.csv > $OUT/$1.txt && cat $OUT/$1.txt
  }
  run sq1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" &&
  run sq2 "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU" &&
  run tcc "TCC_HIT_sum TCC_MISS_sum" && run fetch "FETCH_SIZE" && run write "WRITE_SIZE";;
ab)
  R=$1; W=$2; shift 2
  for r in $(seq 1 $R); do
    for v in product "$@"; do
      if [ $v = product ]; then L=$PWD/testground_amd/libtgsim.so; else L=$PWD/testground_amd/libtgsim_$v.so; fi
      NB=""; [ "$W" = storm ] && NB="--no-beside"
      TGSIM_LIB=$L timeout -k 10 200 python3 -u bench.py --workload $W --no-cpu-baseline $NB --steps 30 > $OUT/${W}_${v}_$r.log 2>&1 || { echo FAIL $v; tail -5 $OUT/${W}_${v}_$r.log; exit 1; }
      python3 -c "import json; j=json.loads(open('$OUT/${W}_${v}_$r.log').read().strip().splitlines()[-1]); print('$v', 'round $r', j['value'], 'msgs/s', round(j['ms_per_step'],5), 'ms/step', ' '.join('%s=%.1f' % (k, v['avg_us']) for k, v in sorted(j['kernels_probe'].items())))"
    done
  done;;
*) echo "usage: tools/gpu.sh tests|bench|evidence|pmc|ab <out> ..."; exit 2;;
esac
