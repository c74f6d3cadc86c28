#!/bin/bash
# PMC passes for one kernel (run on the GPU box): tools/pmc.sh <kernel-regex> <outdir> [bench args...]
# One rocprofv3 run per counter group (the hardware cannot split groups over passes).
set -o pipefail
K=${1:-k_chain_grp}; OUT=${2:-gpurun_out/pmc}; shift 2
mkdir -p $OUT
export TMPDIR=/tmp
ARGS=${@:-"--ranks-per-gpu 8 --streams 1 --max-batches 1 --steps 1 --warmup 0 --cpu-baseline 0 --verify 0 --host-io 0 --solo 0"}
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_LEVEL_WAVES" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_VALU"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set --kernel-include-regex "$K" -d $OUT/p$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT
