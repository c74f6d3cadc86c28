# Config 5 on one GPU box: replay tests, then the streaming decode bench at 4 and 8 contexts.
set -o pipefail
mkdir -p gpurun_out/r3
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_replay.py tests/test_gpu_parity.py tests/test_gzip_stage.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3/pytest.log 2>&1 || { tail -40 gpurun_out/r3/pytest.log; exit 1; }
tail -3 gpurun_out/r3/pytest.log
for S in 4 8; do
timeout -k 10 400 python -u tools/replay_bench.py --ranks 4096 --events 100000 --streams $S > gpurun_out/r3/replay_s$S.json 2> gpurun_out/r3/replay_s$S.err || { tail -30 gpurun_out/r3/replay_s$S.err; exit 1; }
cat gpurun_out/r3/replay_s$S.json
done
timeout -k 10 400 python -u tools/replay_bench.py --ranks 4096 --events 100000 --streams 8 --py-sink > gpurun_out/r3/replay_pysink.json 2> gpurun_out/r3/replay_pysink.err || { tail -30 gpurun_out/r3/replay_pysink.err; exit 1; }
cat gpurun_out/r3/replay_pysink.json
