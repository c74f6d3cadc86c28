# Lanes and hardware queues: tools/queues2.sh <tag> "<queues> <streams>" ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
i=0
for QS in "$@"; do
  set -- $QS; Q=$1; S=$2; i=$((i+1))
  case "$Q" in ""|*[!0-9]*) echo "queues must be a number from 1 to 32, got '$Q'"; exit 2;; esac
  if [ "$Q" -lt 1 ] || [ "$Q" -gt 32 ]; then echo "queues must be from 1 to 32 (the box refuses more), got $Q"; exit 2; fi
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 200 python -u bench.py --cpu-baseline 0 --host-io 0 --solo 0 --steps 6 --max-batches 2 --streams $S > $OUT/r$i.json 2> $OUT/r$i.err || { tail -20 $OUT/r$i.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/r$i.json')); print('queues $Q streams $S:', d['value'], 'GB/s', d['ms_per_step'], 'ms', 'verify_failures', d['config']['verify_failures'])"
done
