# Resident rank traces per batch: tools/ranks_ab.sh <tag> <ranks>...
set -o pipefail
OUT=gpurun_out/$1; shift; mkdir -p $OUT
export TMPDIR=/tmp
for R in "$@"; do
  timeout -k 10 300 python -u bench.py --cpu-baseline 0 --host-io 0 --solo 0 --steps ${STEPS:-8} --max-batches ${BATCHES:-1} --ranks-per-gpu $R > $OUT/r$R.json 2> $OUT/r$R.err || { tail -20 $OUT/r$R.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/r$R.json')); c=d['config']; print('ranks/batch $R:', d['value'], 'GB/s', d['ms_per_step'], 'ms', 'HBM', c['hbm_used_gb'], 'of', c['hbm_total_gb'], 'verify_failures', c['verify_failures'])"
done
