#!/bin/bash
# Lane phase offset x chain grid.  tools/stagger_grid.sh <tag> <grid:stagger_ms>...
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
for gv in "$@"; do
  g=${gv%%:*}; v=${gv##*:}
  CDCX_CHAIN_GRID=$g CDCX_BENCH_STAGGER_MS=$v timeout -k 10 300 python -u bench.py --max-batches 1 --steps 16 --warmup 1 --solo 0 --cpu-baseline 0 --host-io 0 --verify 0 > $OUT/g${g}_st$v.json 2> $OUT/g${g}_st$v.err || { tail -20 $OUT/g${g}_st$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/g${g}_st$v.json'));print('grid $g stagger $v ms:',d['value'],'GB/s',d['ms_per_step'],'ms/step')"
done
