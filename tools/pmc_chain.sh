#!/bin/bash
# PMC passes for one kernel (run on the GPU box): tools/pmc_chain.sh <kernel-regex> <outdir>
set -e
K=${1:-k_chain_seg}; OUT=${2:-gpurun_out/pmc}
mkdir -p $OUT
export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
BENCH="python3 bench.py --ranks-per-gpu 8 --steps 1 --warmup 0 --cpu-baseline 0 --verify-ranks 0"
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "$K" -d $OUT/p$i -o run --output-format csv -- $BENCH > $OUT/p$i.log 2>&1
done
echo done
