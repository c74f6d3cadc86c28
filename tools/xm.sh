# ablation timings (diagnostics): tools/xm.sh <ENVVAR> <modes...>
V=$1; shift
for m in "$@"; do
  env $V=$m timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --cpu-baseline 0 --verify-ranks 0 --host-io 0 --streams 1 --ranks-per-gpu 32 --kernel-report 2>&1 | grep -E "chain_grp|perm_grp" | sed "s/^/mode $m /"
done
