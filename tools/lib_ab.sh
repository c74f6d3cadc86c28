# A/B of library builds on one batch over 12 steps and two batches over 3: tools/lib_ab.sh <tag> <lib.so>...
set -o pipefail
OUT=gpurun_out/$1; shift; mkdir -p $OUT
export TMPDIR=/tmp
for L in "$@"; do
  N=$(basename $L .so)
  CDCX_LIB=$L timeout -k 10 200 python -u bench.py --cpu-baseline 0 --host-io 0 --solo 0 --steps 12 --max-batches 1 --verify 0 > $OUT/$N.b12.json 2> $OUT/$N.b12.err || { tail -20 $OUT/$N.b12.err; exit 1; }
  CDCX_LIB=$L timeout -k 10 200 python -u bench.py --cpu-baseline 0 --host-io 0 --solo 0 --steps 3 --max-batches 2 > $OUT/$N.b3.json 2> $OUT/$N.b3.err || { tail -20 $OUT/$N.b3.err; exit 1; }
  python -c "import json; a=json.load(open('$OUT/$N.b12.json')); b=json.load(open('$OUT/$N.b3.json')); print('$N: 12 steps', a['value'], 'GB/s; 3 steps x 2 batches', b['value'], 'GB/s, verify_failures', b['config']['verify_failures'])"
done
