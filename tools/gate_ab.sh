# A/B of the gates of the issue-bound kernels: tools/gate_ab.sh <tag> <mode:chain_depth:perm_depth>...
set -o pipefail
OUT=gpurun_out/$1; shift; mkdir -p $OUT
export TMPDIR=/tmp
for M in "$@"; do
  IFS=: read mode cd pd <<< "$M"
  CDCX_GATE=$mode CDCX_GATE_CHAIN=$cd CDCX_GATE_PERM=$pd timeout -k 10 200 python -u bench.py --cpu-baseline 0 --host-io 0 --solo 0 --steps ${STEPS:-12} --max-batches ${BATCHES:-1} --verify ${VERIFY:-0} > $OUT/g_$mode-$cd-$pd.json 2> $OUT/g_$mode-$cd-$pd.err || { tail -20 $OUT/g_$mode-$cd-$pd.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/g_$mode-$cd-$pd.json')); print('gate mode $mode chain depth $cd perm depth $pd:', d['value'], 'GB/s', d['ms_per_step'], 'ms')"
done
