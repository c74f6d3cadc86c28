#!/bin/bash
# Timing of several in-tree builds of the library on one box, interleaved twice:
#   LIBS="libcdcx_a.so libcdcx.so" tools/ab.sh <tag> [bench args...]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
for i in 1 2; do
  for L in $LIBS; do
    CDCX_LIB=$L timeout -k 10 300 python -u bench.py --kernel-report "$@" > $OUT/$L.$i.json 2> $OUT/$L.$i.err || { echo "bench $L failed"; tail -20 $OUT/$L.$i.err; exit 1; }
    echo "$L $i $(python3 -c "import json,sys;print(json.load(open('$OUT/$L.$i.json'))['value'])")"
  done
done
