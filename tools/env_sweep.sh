#!/bin/bash
# Whole-path throughput under settings of one environment knob (run on the GPU box):
# tools/env_sweep.sh <outdir> <VAR> <value> [value...]   (two batches, 4 lanes)
set -o pipefail
OUT=$1; VAR=$2; shift 2
mkdir -p $OUT
for v in "$@"; do
  env $VAR=$v timeout -k 10 300 python -u bench.py --max-batches 2 --steps 3 --warmup 1 --solo 0 --cpu-baseline 0 --host-io 0 > $OUT/${VAR}_$v.json 2> $OUT/${VAR}_$v.err || { tail -20 $OUT/${VAR}_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/${VAR}_$v.json'));print('$VAR=$v:',d['value'],'GB/s',d['ms_per_step'],'ms/step verify_failures',d['config']['verify_failures'])"
done
