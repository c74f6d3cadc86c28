#!/bin/bash
# One GPU-box pass: parity tests, bench, rocprofv3 kernel stats of the default (4-lane) run and of
# a one-lane run (the kernel durations that the bench's roofline.launch_ms must agree with).
# tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-run}; OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 400 python -u bench.py --kernel-report > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --max-batches 2 --cpu-baseline 0 --host-io 0 --solo 0 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof.log; exit 1; }
cp $OUT/prof/run_kernel_stats.csv $OUT/kernel_stats.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_solo -o run --output-format csv -- python3 bench.py --streams 1 --ranks-per-gpu 32 --steps 3 --warmup 1 --max-batches 1 --cpu-baseline 0 --host-io 0 --solo 0 > $OUT/prof_solo.log 2>&1 || { echo "rocprof (one lane) failed"; tail -30 $OUT/prof_solo.log; exit 1; }
cp $OUT/prof_solo/run_kernel_stats.csv $OUT/solo_kernel_stats.csv
head -8 $OUT/solo_kernel_stats.csv | cut -c1-200
