# Config 5 at 1 M events/rank, 1024 ranks: A/B of library builds on one box.  tools/replay_lib_ab.sh <tag> <lib>...
set -o pipefail
OUT=gpurun_out/$1; shift; mkdir -p $OUT
export TMPDIR=/tmp
for L in "$@"; do
  N=$(basename $L .so)
  CDCX_LIB=$L timeout -k 10 600 python -u tools/replay_bench.py --ranks 1024 --events 1000000 --streams 4 --tables --gen-batch 128 > $OUT/replay_$N.json 2> $OUT/replay_$N.err || { tail -30 $OUT/replay_$N.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/replay_$N.json')); print('$N:', d['seconds'], 's', d['record_gbps'], 'GB/s of records', d['thread_s'])"
done
