# A/B of the 16-lane chain tier's grid (CDCX_CHAIN_GRID) on the bench configuration, after
# the chain tier parity tests.  tools/grid_ab.sh <tag> <grid>...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "chain or batch or generator_workloads" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for G in "$@"; do
  CDCX_CHAIN_GRID=$G timeout -k 10 300 python -u bench.py --cpu-baseline 0 --host-io 0 --steps 4 > $OUT/bench_g$G.json 2> $OUT/bench_g$G.err || { tail -20 $OUT/bench_g$G.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/bench_g$G.json')); print('grid $G', d['value'], d['ms_per_step'])"
done
