# Lanes per batch: tools/streams_ab.sh <tag> <streams>...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for S in "$@"; do
  timeout -k 10 200 python -u bench.py --cpu-baseline 0 --host-io 0 --solo 0 --steps 6 --max-batches 2 --streams $S > $OUT/s$S.json 2> $OUT/s$S.err || { tail -20 $OUT/s$S.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/s$S.json')); print('streams $S:', d['value'], 'GB/s', d['ms_per_step'], 'ms', 'verify_failures', d['config']['verify_failures'])"
done
