# Config 5 on one GPU box: replay tests, then the streaming decode bench (tools/replay_gpu.sh [tag]).
set -o pipefail
OUT=gpurun_out/${1:-r02_replay}
mkdir -p $OUT
export TMPDIR=/tmp
df -h /tmp /dev/shm | tee $OUT/df.txt
timeout -k 10 300 python -u -m pytest tests/test_replay.py tests/test_chunk_api.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
# small files (100 K events/rank): dumps vs flat tables
timeout -k 10 400 python -u tools/replay_bench.py --ranks 4096 --events 100000 --streams 4 > $OUT/replay_100k_dumps.json 2> $OUT/replay_100k_dumps.err || { tail -30 $OUT/replay_100k_dumps.err; exit 1; }
cat $OUT/replay_100k_dumps.json
timeout -k 10 400 python -u tools/replay_bench.py --ranks 4096 --events 100000 --streams 4 --tables > $OUT/replay_100k_tables.json 2> $OUT/replay_100k_tables.err || { tail -30 $OUT/replay_100k_tables.err; exit 1; }
cat $OUT/replay_100k_tables.json
# 1 M events/rank: as many ranks of the 4096 as the scratch disk holds (15 MB per file)
FREE_GB=$(df --output=avail -BG /tmp | tail -1 | tr -dc 0-9)
RANKS=4096; [ "$FREE_GB" -lt 90 ] && RANKS=1024; [ "$FREE_GB" -lt 25 ] && RANKS=256
echo "free ${FREE_GB}G -> $RANKS ranks x 1M events"
timeout -k 10 800 python -u tools/replay_bench.py --ranks $RANKS --events 1000000 --streams 4 --tables --gen-batch 128 > $OUT/replay_1m_tables.json 2> $OUT/replay_1m_tables.err || { tail -30 $OUT/replay_1m_tables.err; exit 1; }
cat $OUT/replay_1m_tables.json
