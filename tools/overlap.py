"""Concurrency of kernels in a rocprofv3 kernel trace (several streams): per kernel, total
time, and the time-weighted number of kernels running beside it.
usage: python tools/overlap.py run_kernel_trace.csv [t0_frac]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = []
for r in rows:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("cdcx::", "")
    if n.startswith("k_gen") or "rocclr" in n:
        continue
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n))
ev.sort()
t0 = ev[0][0] + (ev[-1][1] - ev[0][0]) * (float(sys.argv[2]) if len(sys.argv) > 2 else 0.0)
ev = [e for e in ev if e[0] >= t0]
# sweep
pts = sorted([(s, 1, n) for s, e, n in ev] + [(e, -1, n) for s, e, n in ev])
run = collections.Counter()
tot = collections.Counter()
conc = collections.Counter()
busy = 0.0
last = pts[0][0]
for t, d, n in pts:
    dt = t - last
    k = sum(run.values())
    if k:
        busy += dt
        for m, c in run.items():
            if c:
                tot[m] += dt * c
                conc[m] += dt * c * (k - 1)
    run[n] += d
    last = t
span = pts[-1][0] - pts[0][0]
print(f"span {span/1e6:.1f} ms, busy {busy/1e6:.1f} ms, kernel-time {sum(tot.values())/1e6:.1f} ms")
for m, v in tot.most_common(20):
    print(f"  {m:24s} {v/1e6:8.2f} ms  beside {conc[m]/max(v,1):.2f}")
