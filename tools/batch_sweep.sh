#!/bin/bash
# Throughput against the batch size per lane (run on the GPU box):
# tools/batch_sweep.sh <outdir> "<ranks-per-gpu>:<streams> ..."
set -o pipefail
OUT=${1:-gpurun_out/sweep}; shift
mkdir -p $OUT
for cfg in ${@:-"32:4 96:4"}; do
  R=${cfg%%:*}; S=${cfg##*:}
  timeout -k 10 300 python -u bench.py --ranks-per-gpu $R --streams $S --max-batches $(( 192 / R )) --steps 3 --warmup 1 --solo 0 --cpu-baseline 0 --host-io 0 > $OUT/b_${R}_${S}.json 2> $OUT/b_${R}_${S}.err || { tail -20 $OUT/b_${R}_${S}.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/b_${R}_${S}.json'));print('$R ranks/batch on $S lanes:',d['value'],'GB/s',d['ms_per_step'],'ms/step verify_failures',d['config']['verify_failures'])"
done
