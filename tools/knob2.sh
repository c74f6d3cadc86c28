# A/B of library env settings on two batches of the bench: tools/knob2.sh <tag> "VAR=v VAR2=w" "..." ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
i=0
for SET in "$@"; do
  i=$((i+1))
  env $SET timeout -k 10 200 python -u bench.py --cpu-baseline 0 --host-io 0 --solo ${SOLO:-0} --steps ${STEPS:-6} --max-batches 2 --kernel-report > $OUT/s$i.json 2> $OUT/s$i.err || { tail -20 $OUT/s$i.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/s$i.json')); print('$SET:', d['value'], 'GB/s', d['ms_per_step'], 'ms', 'verify_failures', d['config']['verify_failures'])"
  grep -E "${SHOW:-k_scatter|k_chain_exits}" $OUT/s$i.err
done
