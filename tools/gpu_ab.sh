#!/bin/bash
# A/B timing of experiment builds against the product build on one box, interleaved:
#   tools/gpu_ab.sh <outdir> <rounds> <workload> <name>...   (names of testground_amd/libtgsim_<name>.so)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-ab}; R=${2:-2}; W=${3:-storm}; shift 3
mkdir -p $OUT
for r in $(seq 1 $R); do
  for v in product "$@"; do
    if [ $v = product ]; then L=$PWD/testground_amd/libtgsim.so; else L=$PWD/testground_amd/libtgsim_$v.so; fi
    TGSIM_LIB=$L timeout -k 10 200 python3 -u bench.py --workload $W --no-cpu-baseline --steps 30 > $OUT/${W}_${v}_$r.log 2>&1 || { echo FAIL $v; tail -5 $OUT/${W}_${v}_$r.log; exit 1; }
    python3 -c "import json,sys; j=json.loads(open('$OUT/${W}_${v}_$r.log').read().strip().splitlines()[-1]); print('$v', 'round $r', round(j['value']/1e9,4), 'e9/s', round(j['ms_per_step'],5), 'ms/step')"
  done
done
