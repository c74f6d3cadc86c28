# Config 5 at 1 M events/rank, 1024 ranks, with and without the gates.  tools/replay_quick.sh <tag>
set -o pipefail
OUT=gpurun_out/${1:-rq}; mkdir -p $OUT
export TMPDIR=/tmp
for G in 11 0; do
  CDCX_GATE=$G timeout -k 10 600 python -u tools/replay_bench.py --ranks 1024 --events 1000000 --streams 4 --tables --gen-batch 128 > $OUT/replay_1m_g$G.json 2> $OUT/replay_1m_g$G.err || { tail -30 $OUT/replay_1m_g$G.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/replay_1m_g$G.json')); print('CDCX_GATE=$G:', d['seconds'], 's', d['record_gbps'], 'GB/s of records', d['thread_s'])"
done
