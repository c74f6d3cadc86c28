# Engine / memory clocks and power sampled twice a second while the bench runs.  tools/clock_watch.sh <tag>
set -o pipefail
TAG=${1:-clk}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u bench.py --cpu-baseline 0 --host-io 0 --solo 0 --steps 6 --max-batches 2 > $OUT/bench.json 2> $OUT/bench.err &
BP=$!
for i in $(seq 1 120); do
  kill -0 $BP 2>/dev/null || break
  (date +%s.%N; rocm-smi --showclocks --showpower --showuse 2>&1 | grep -E "sclk|mclk|fclk|Power|GPU use|busy") >> $OUT/smi.txt
  sleep 0.5
done
wait $BP || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], 'GB/s')"
grep -E "sclk" $OUT/smi.txt | sort | uniq -c | sort -rn | head -12
grep -E "Power" $OUT/smi.txt | sort | uniq -c | sort -rn | head -8
