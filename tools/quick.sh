# Parity tests of the encode/decode kernels, then the bench on one batch over 12 steps (steady
# state) and on two batches over 3.  tools/quick.sh <tag> [VAR=value ...]
set -o pipefail
OUT=gpurun_out/$1; shift; mkdir -p $OUT
export TMPDIR=/tmp
for kv in "$@"; do export "$kv"; done
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_config3_full.py tests/test_zz_no_alloc.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python -u bench.py --cpu-baseline 0 --host-io 0 --solo 0 --steps 12 --max-batches 1 --verify 0 > $OUT/b12.json 2> $OUT/b12.err || { tail -20 $OUT/b12.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/b12.json')); print('12 steps, 1 batch:', d['value'], 'GB/s', d['ms_per_step'], 'ms')"
timeout -k 10 200 python -u bench.py --cpu-baseline 0 --host-io 0 --solo 2 --steps 3 --max-batches 2 --kernel-report > $OUT/b3.json 2> $OUT/b3.err || { tail -20 $OUT/b3.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/b3.json')); print('3 steps, 2 batches:', d['value'], 'GB/s', d['ms_per_step'], 'ms', 'verify_failures', d['config']['verify_failures'])"
head -12 $OUT/b3.err
