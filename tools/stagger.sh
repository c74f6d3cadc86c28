#!/bin/bash
# Does a phase offset between the lanes help?  One batch, many steps, lane k delayed by k * ms.
set -o pipefail
OUT=$1; shift
mkdir -p $OUT
for v in "$@"; do
  CDCX_BENCH_STAGGER_MS=$v timeout -k 10 300 python -u bench.py --max-batches 1 --steps 16 --warmup 1 --solo 0 --cpu-baseline 0 --host-io 0 --verify 0 > $OUT/st_$v.json 2> $OUT/st_$v.err || { tail -20 $OUT/st_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/st_$v.json'));print('stagger $v ms:',d['value'],'GB/s',d['ms_per_step'],'ms/step')"
done
