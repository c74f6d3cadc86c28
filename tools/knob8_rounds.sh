# tools/knob_rounds.sh with 8 lanes on 8 hardware queues: tools/knob8_rounds.sh <tag> <rounds> <"VAR=v [VAR=v]" | ->...
set -o pipefail
OUT=gpurun_out/$1; shift; R=$1; shift; mkdir -p $OUT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
for r in $(seq 1 $R); do
  i=0
  for E in "$@"; do
    i=$((i+1)); S="$E"; [ "$E" = "-" ] && S="CDCX_NONE=0"
    env $S timeout -k 10 200 python -u bench.py --cpu-baseline 0 --host-io 0 --solo 0 --steps 12 --max-batches 1 --verify 0 --streams ${STREAMS:-8} > $OUT/k$i.$r.json 2> $OUT/k$i.$r.err || { tail -20 $OUT/k$i.$r.err; exit 1; }
    python -c "import json; a=json.load(open('$OUT/k$i.$r.json')); print('[$E] round $r:', a['value'], 'GB/s', a['ms_per_step'], 'ms')" | tee -a $OUT/summary.txt
  done
done
