# Parity tests of the codec kernels, then VALU / SALU / LDS counts and the duration of the kernels
# matching a regex on an 8-rank batch.  tools/pmc_one.sh <tag> <kernel regex>
set -o pipefail
OUT=gpurun_out/$1; K=$2; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_config3_full.py tests/test_zz_no_alloc.py tests/test_corrupt.py tests/test_replay.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
ARGS="--ranks-per-gpu 8 --streams 1 --max-batches 1 --steps 1 --warmup 0 --cpu-baseline 0 --verify 0 --host-io 0 --solo 0"
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --kernel-include-regex "$K" -d $OUT/p1 -o run --output-format csv -- python3 bench.py $ARGS > $OUT/p1.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/p1.log; exit 1; }
python3 - $OUT/p1/run_counter_collection.csv <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.Counter())
for r in csv.DictReader(open(sys.argv[1])):
    acc[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in acc.items():
    print(k, {n: f"{v / 1e6:.1f}M" for n, v in c.items()})
PY
timeout -k 10 200 python -u bench.py --cpu-baseline 0 --host-io 0 --solo 2 --steps 3 --max-batches 2 --kernel-report > $OUT/b3.json 2> $OUT/b3.err || { tail -20 $OUT/b3.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/b3.json')); print('3 steps, 2 batches:', d['value'], 'GB/s', d['ms_per_step'], 'ms', 'verify_failures', d['config']['verify_failures'])"
grep -E "$K" $OUT/b3.err
