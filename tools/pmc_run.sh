#!/bin/bash
# PMC passes over a short storm run (one rocprofv3 invocation per counter group).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc
mkdir -p $OUT
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex "${KREGEX:-k_shape|k_gen_storm|k_extract}" -d $OUT/p$i -o run --output-format csv -- python3 -u tools/probe.py 100000 14 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  echo "pass $i ok: $grp"
done
