# Alternating A/B of lanes per batch (with enough hardware queues for each): tools/streams_rounds.sh <tag> <rounds> <streams>...
set -o pipefail
OUT=gpurun_out/$1; shift; R=$1; shift; mkdir -p $OUT
export TMPDIR=/tmp
for r in $(seq 1 $R); do
  for S in "$@"; do
    Q=${QUEUES:-4}; [ -z "$QUEUES" ] && [ "$S" -gt 4 ] && Q=8
    GPU_MAX_HW_QUEUES=$Q timeout -k 10 200 python -u bench.py --cpu-baseline 0 --host-io 0 --solo 0 --steps 12 --max-batches 1 --verify 0 --streams $S > $OUT/s$S.$r.json 2> $OUT/s$S.$r.err || { tail -20 $OUT/s$S.$r.err; exit 1; }
    python -c "import json; a=json.load(open('$OUT/s$S.$r.json')); print('streams $S (queues $Q) round $r:', a['value'], 'GB/s', a['ms_per_step'], 'ms')" | tee -a $OUT/summary.txt
  done
done
