for m in 0 1 2 4 8 6 15; do
  CDCX_XMODE=$m timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --cpu-baseline 0 --verify-ranks 0 --kernel-report 2>&1 | grep perm_grp | sed "s/^/mode $m /"
done
