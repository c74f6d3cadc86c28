#!/bin/bash
# One rocprofv3 --pmc pass per counter group over EVERY kernel of a small bench run (run on the
# GPU box): tools/pmc_all.sh <outdir> [bench args...]; summary by tools/pmc_table.py (per record
# of the default 8 ranks x 10 M events; PMC_RECORDS overrides the count).
set -o pipefail
OUT=${1:-gpurun_out/pmc_all}; shift 1
mkdir -p $OUT
export TMPDIR=/tmp
ARGS=${@:-"--ranks-per-gpu 8 --streams 1 --max-batches 1 --steps 1 --warmup 0 --cpu-baseline 0 --verify 0 --host-io 0 --solo 0"}
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set -d $OUT/p$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_table.py $OUT ${PMC_RECORDS:-80000000} $OUT/pmc_traffic.json
