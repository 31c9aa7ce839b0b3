#!/bin/bash
# Topic fan-out (tools/bench_topics.py): the timed fill, then one rocprofv3 pass of WRITE_SIZE and one of
# FETCH_SIZE over the fill kernel, so the quoted store rate is backed by the bytes the counters saw
# (VERDICT r2 item 8).   tools/gpu_topics_pmc.sh <outdir-under-gpurun_out> [n]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-topics}
N=${2:-100000}
mkdir -p $OUT
timeout -k 10 240 python3 -u tools/bench_topics.py --n $N --reps 5 > $OUT/topics_fanout.jsonl 2> $OUT/topics_fanout.err || { echo TOPICS_FAIL; tail -20 $OUT/topics_fanout.err; exit 1; }
cat $OUT/topics_fanout.jsonl
for c in WRITE_SIZE FETCH_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace -d $OUT/pmc_$c -o run --output-format csv \
    -- python3 -u tools/bench_topics.py --n $N --reps 1 > $OUT/pmc_$c.log 2>&1 || { echo PMC_FAIL $c; tail -20 $OUT/pmc_$c.log; exit 1; }
done
python3 tools/topics_pmc_summary.py $OUT $N | tee $OUT/topics_pmc.json
