# tools/lib_ab2.sh on the bench's default lanes (8 lanes, 8 hardware queues): tools/lib_ab8.sh <tag> <rounds> <lib.so>...
set -o pipefail
OUT=gpurun_out/$1; shift; R=$1; shift; mkdir -p $OUT
export TMPDIR=/tmp
for r in $(seq 1 $R); do
  for L in "$@"; do
    N=$(basename $L .so)
    CDCX_LIB=$L timeout -k 10 200 python -u bench.py --cpu-baseline 0 --host-io 0 --solo 0 --steps ${STEPS:-12} --max-batches ${BATCHES:-1} --verify 0 > $OUT/$N.$r.json 2> $OUT/$N.$r.err || { tail -20 $OUT/$N.$r.err; exit 1; }
    python -c "import json; a=json.load(open('$OUT/$N.$r.json')); print('$N round $r:', a['value'], 'GB/s', a['ms_per_step'], 'ms')" | tee -a $OUT/summary.txt
  done
done
