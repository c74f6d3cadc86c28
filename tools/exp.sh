#!/bin/bash
# Quick kernel experiment on the GPU box: the tier / parity tests that cover the chain,
# rank and permutation kernels, then one single-stream batch with per-kernel times
# (a launch alone on the GPU).  tools/exp.sh <tag> [pytest -k expression]
set -o pipefail
TAG=${1:-exp}; K=${2:-"tiers or batch_encode or generator_workloads or random_streams"}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "$K" --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
timeout -k 10 200 python -u bench.py --ranks-per-gpu 24 --streams 1 --max-batches 1 --steps 3 --warmup 1 --solo 0 --cpu-baseline 0 --host-io 0 --kernel-report > gpurun_out/$TAG/bench1.json 2> gpurun_out/$TAG/bench1.err || { tail -30 gpurun_out/$TAG/bench1.err; exit 1; }
head -24 gpurun_out/$TAG/bench1.err | tail -23; tail -1 gpurun_out/$TAG/bench1.err
python3 -c "import json;d=json.load(open('gpurun_out/$TAG/bench1.json'));print('1 stream:',d['value'],'GB/s verify',d['config']['verify'])"
