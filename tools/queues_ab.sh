# A/B of the number of HIP hardware queues per process (GPU_MAX_HW_QUEUES, HIP's default 4) against
# the number of lanes of a batch.  tools/queues_ab.sh <tag> <queues:streams>...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for QS in "$@"; do
  Q=${QS%%:*}; S=${QS##*:}
  case "$Q" in ""|*[!0-9]*) echo "queues must be a number from 1 to 32, got '$Q'"; exit 2;; esac
  if [ "$Q" -lt 1 ] || [ "$Q" -gt 32 ]; then echo "queues must be from 1 to 32 (the box refuses more), got $Q"; exit 2; fi
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 200 python -u bench.py --cpu-baseline 0 --host-io 0 --solo 0 --steps 3 --max-batches 2 --streams $S > $OUT/q${Q}_s${S}.json 2> $OUT/q${Q}_s${S}.err || { tail -20 $OUT/q${Q}_s${S}.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/q${Q}_s${S}.json')); print('queues $Q streams $S:', d['value'], 'GB/s', d['ms_per_step'], 'ms', 'verify_failures', d['config']['verify_failures'])"
done
