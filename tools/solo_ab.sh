# Per-kernel times of one lane alone, per library build: tools/solo_ab.sh <tag> <lib.so>...   (paths relative to rempi_amd/)
set -o pipefail
OUT=gpurun_out/$1; shift; mkdir -p $OUT
export TMPDIR=/tmp
for L in "$@"; do
  N=$(basename $L .so)
  CDCX_LIB=$L timeout -k 10 200 python -u bench.py --cpu-baseline 0 --host-io 0 --solo 4 --steps 2 --max-batches 1 --verify 0 --kernel-report > $OUT/$N.json 2> $OUT/$N.err || { tail -20 $OUT/$N.err; exit 1; }
  echo "== $N"; grep "alone" $OUT/$N.err | sort -k8 -n -r | head -${TOP:-12}
done
