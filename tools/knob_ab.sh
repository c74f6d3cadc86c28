# A/B of one library env knob on two batches of the bench.  tools/knob_ab.sh <tag> <VAR> <value>...
set -o pipefail
TAG=$1; VAR=$2; shift; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for V in "$@"; do
  env $VAR=$V timeout -k 10 200 python -u bench.py --cpu-baseline 0 --host-io 0 --solo 0 --steps 3 --max-batches 2 ${BENCH_ARGS:-} > $OUT/${VAR}_$V.json 2> $OUT/${VAR}_$V.err || { tail -20 $OUT/${VAR}_$V.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/${VAR}_$V.json')); print('$VAR=$V:', d['value'], 'GB/s', d['ms_per_step'], 'ms', 'verify_failures', d['config']['verify_failures'])"
done
