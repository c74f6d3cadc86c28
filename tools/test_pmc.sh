# GPU parity tests, a two-batch bench, then the PMC passes of every kernel.  tools/test_pmc.sh <tag>
set -o pipefail
TAG=${1:-tp}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --host-io 0 --max-batches 2 --kernel-report > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], 'GB/s', d['ms_per_step'], 'ms', 'verify_failures', d['config']['verify_failures'])"
head -24 $OUT/bench.err
bash tools/pmc_all.sh $OUT/pmc > $OUT/pmc_table.txt 2>&1 || { tail -20 $OUT/pmc_table.txt; exit 1; }
head -24 $OUT/pmc_table.txt; tail -1 $OUT/pmc_table.txt
