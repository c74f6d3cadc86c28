#!/bin/bash
# bench variants on the GPU box: tools/gpu_bench.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-b}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u bench.py --kernel-report "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
