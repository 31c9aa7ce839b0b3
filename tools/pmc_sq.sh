#!/bin/bash
# SQ cycle breakdown (one rocprofv3 --pmc pass) of every storm kernel over a short probe run.
#   tools/pmc_sq.sh <outdir>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-sq}
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES \
  -d $OUT/p1 -o run --output-format csv -- python3 -u tools/probe.py 100000 14 > $OUT/p1.log 2>&1 || { echo "pass 1 failed"; tail $OUT/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU GRBM_GUI_ACTIVE \
  -d $OUT/p2 -o run --output-format csv -- python3 -u tools/probe.py 100000 14 > $OUT/p2.log 2>&1 || { echo "pass 2 failed"; tail $OUT/p2.log; exit 1; }
python3 tools/pmc_summary.py $(find $OUT -name '*counter_collection.csv') > $OUT/summary.txt
cat $OUT/summary.txt
