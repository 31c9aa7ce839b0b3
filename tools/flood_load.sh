#!/bin/bash
# Config 5 at heavier publication loads (VERDICT r5 "missing" item 4): P floods per wave (one wave
# every 4 windows), P = 1, 2, 4, each its own bench run (GPU box, under gpurun). From P = 2 the
# 1-Mbit/s senders are overloaded (8 forwards x 512 B per flood every 40 ms against 5 KB drained):
# their netem queues fill to the 1000-packet limit and the wheel holds their backlog, so the arena
# (2 x max_records) is sized per P:
#   bash tools/flood_load.sh <out>   ->  gpurun_out/<out>/flood_p<P>.log and a summary line each
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; mkdir -p $O
for P in 1 2 4; do
  R=$((1 << 25)); [ $P -eq 2 ] && R=$((1 << 26)); [ $P -eq 4 ] && R=$((1 << 27))
  timeout -k 10 400 python3 -u bench.py --workload flood --pubs-per-wave $P --flood-records-per-pub $R \
    --no-cpu-baseline > $O/flood_p$P.log 2>&1 || { echo "P=$P failed"; tail -5 $O/flood_p$P.log; exit 1; }
  python3 -c "import json; j=json.loads(open('$O/flood_p$P.log').read().strip().splitlines()[-1]); print('pubs_per_wave $P', 'records_per_pub $R', '%.3e' % j['value'], 'msgs/s', round(j['ms_per_step'], 4), 'ms/window', j['config']['delivered_in_timed_steps'], 'delivered in', j['steps'], 'windows; frac', round(j['roofline']['frac'], 4), 'dominant', j['roofline'].get('kernel'))"
done
