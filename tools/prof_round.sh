#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run, then PMC passes (one rocprofv3 run each).
#   tools/prof_round.sh <outdir-under-gpurun_out> [pmc group ...]
set -o pipefail
OUT=gpurun_out/${1:-prof}
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv \
  -- python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 10 > $OUT/bench_trace.log 2>&1 || { echo TRACE_FAIL; tail -5 $OUT/bench_trace.log; exit 1; }
python3 tools/trace_summary.py $OUT/trace/run_kernel_trace.csv --last 20 > $OUT/trace_summary.txt 2>&1
head -30 $OUT/trace_summary.txt
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "${KREGEX:-k_tb_bucket|k_emit_bucket|k_shape|k_wheel_scatter|k_extract|k_gen_storm|k_bkt}" \
    -d $OUT/pmc$i -o run --output-format csv -- python3 -u bench.py --no-cpu-baseline --steps 5 --warmup 5 > $OUT/pmc$i.log 2>&1 \
    || { echo "pmc pass $i failed: $grp"; tail -3 $OUT/pmc$i.log; exit 1; }
  echo "pmc pass $i ok: $grp"
done
