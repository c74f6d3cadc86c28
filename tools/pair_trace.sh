# Two lanes, offset in phase, under rocprofv3 --kernel-trace.  tools/pair_trace.sh <tag> <stagger ms>
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
export TMPDIR=/tmp
export CDCX_BENCH_STAGGER_MS=${2:-20}
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof -o run --output-format csv -- python3 bench.py --streams 2 --ranks-per-gpu 48 --max-batches 1 --steps 8 --warmup 1 --solo 2 --cpu-baseline 0 --host-io 0 --verify 0 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 tools/pair_overlap.py $OUT/prof/run_kernel_trace.csv | head -60
