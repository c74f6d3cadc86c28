"""Pairwise co-run slowdowns from a rocprofv3 kernel trace of a two-lane run: for every kernel
launch X whose duration is covered (>= 85 %) by launches of ONE other kernel name Y and by
nothing else for more than 10 %, X's duration against its duration alone (launches with
< 5 % overlap).  usage: python tools/pair_overlap.py run_kernel_trace.csv"""
import collections
import csv
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("cdcx::", "")
    if n.startswith("k_gen") or n.startswith("__amd"):
        continue
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n, r["Stream_Id"]))
rows.sort()
alone = collections.defaultdict(list)
pair = collections.defaultdict(list)
for i, (s, e, n, st) in enumerate(rows):
    d = e - s
    if d < 200_000:
        continue
    ov = collections.Counter()
    for (s2, e2, n2, st2) in rows:
        if st2 == st or e2 <= s or s2 >= e:
            continue
        ov[n2] += min(e, e2) - max(s, s2)
    tot = sum(ov.values())
    if tot < 0.05 * d:
        alone[n].append(d)
        continue
    top, tv = ov.most_common(1)[0]
    if tv >= 0.85 * d and tot - tv <= 0.10 * d:
        pair[(n, top)].append(d)
print(f"{'kernel':18s} {'beside':18s} {'n':>3s} {'ms':>8s} {'alone ms':>9s} {'x':>6s}")
for (n, y), ds in sorted(pair.items(), key=lambda kv: -sum(kv[1])):
    if n not in alone:
        continue
    a = sum(alone[n]) / len(alone[n])
    m = sum(ds) / len(ds)
    print(f"{n:18s} {y:18s} {len(ds):3d} {m / 1e6:8.3f} {a / 1e6:9.3f} {m / a:6.2f}")
