#!/bin/bash
# Storm PMC passes (one counter group per run, as the guide prescribes): SQ stall/occupancy, LDS,
# TCC hit/miss, HBM bytes.   [KR=<kernel regex>] tools/gpu_storm_pmc.sh <outdir> [extra bench args]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-spmc}
shift
mkdir -p $OUT
B="bench.py --no-cpu-baseline --steps 5 --warmup 5 $*"
KR=${KR:-"k_tb_bucket|k_emit_bucket|k_extract_shape|k_wheel_scatter|k_gen_storm|k_bkt_local|k_local_hist|k_window_start"}
run() {
  timeout -s KILL 150 rocprofv3 --pmc $2 --kernel-include-regex "$KR" -d $OUT/$1 -o run --output-format csv \
    -- python3 -u $B > $OUT/$1.log 2>&1 || { echo "PMC_FAIL $1"; tail -5 $OUT/$1.log; exit 1; }
}
run sq1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD"
run sq2 "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU"
run tcc "TCC_HIT_sum TCC_MISS_sum"
run fetch "FETCH_SIZE"
run write "WRITE_SIZE"
for p in sq1 sq2 tcc fetch write; do
  python3 tools/pmc_table.py $OUT/$p/run_counter_collection.csv > $OUT/$p.txt
  cat $OUT/$p.txt
done
