# A/B of library env knobs on the bench configuration, after the GPU parity tests.
# tools/env_ab.sh <tag> <VAR=value | ->...   ("-" = no knob)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
i=0
for E in "$@"; do
  i=$((i+1))
  if [ "$E" = "-" ]; then E="CDCX_NONE=0"; fi
  env $E timeout -k 10 300 python -u bench.py --cpu-baseline 0 --host-io 0 --steps 4 > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { tail -20 $OUT/bench_$i.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$i.json')); print('$E', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 --host-io 0 > $OUT/prof.log 2>&1 || { tail -30 $OUT/prof.log; exit 1; }
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
grep -i "rocclr" $OUT/kernel_stats.csv | cut -c1-120
