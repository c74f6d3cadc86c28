"""Lane overlap from a rocprofv3 --kernel-trace CSV: for the window of the last encode+decode
step of every stream, the time with 0/1/2/... kernels in flight, and per stream the gaps
between consecutive kernels (host round trips and launch latency).

usage: python tools/trace_overlap.py <run_kernel_trace.csv> [steps-from-the-end]"""
import collections
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if not r["Kernel_Name"].startswith("__amd") and "k_gen" not in r["Kernel_Name"]]
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    r["k"] = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("cdcx::", "")
streams = collections.defaultdict(list)
for r in rows:
    streams[r["Stream_Id"]].append(r)
nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
win_s, win_e = 0, 0
sel = []
for sid, rs in streams.items():
    rs.sort(key=lambda r: r["s"])
    starts = [i for i, r in enumerate(rs) if r["k"] == "k_tile_hist"]
    first = starts[-nsteps]
    sel += rs[first:]
    print(f"stream {sid}: {len(rs) - first} kernels in the window, {rs[first]['s']} .. {rs[-1]['e']}")
t0 = min(r["s"] for r in sel)
t1 = max(r["e"] for r in sel)
ev = []
for r in sel:
    ev.append((r["s"], 1))
    ev.append((r["e"], -1))
ev.sort()
depth, last, hist = 0, t0, collections.Counter()
for t, d in ev:
    hist[depth] += t - last
    last = t
    depth += d
tot = t1 - t0
print(f"window {tot / 1e6:.3f} ms")
for d in sorted(hist):
    print(f"  {d} kernels in flight: {hist[d] / 1e6:8.3f} ms  {100 * hist[d] / tot:5.1f}%")
for sid, rs in streams.items():
    rs = [r for r in rs if r["s"] >= t0]
    busy = sum(r["e"] - r["s"] for r in rs)
    gaps = [(rs[i + 1]["s"] - rs[i]["e"], rs[i]["k"], rs[i + 1]["k"]) for i in range(len(rs) - 1)]
    big = sorted(gaps, reverse=True)[:8]
    print(f"stream {sid}: busy {busy / 1e6:.3f} ms, gaps {sum(g[0] for g in gaps) / 1e6:.3f} ms; largest:",
          ", ".join(f"{g[0] / 1e3:.0f}us {g[1]}->{g[2]}" for g in big))
# time per kernel name inside the window, and mean concurrency while it runs
per = collections.defaultdict(lambda: [0, 0])
for r in sel:
    per[r["k"]][0] += r["e"] - r["s"]
    per[r["k"]][1] += 1
print("kernel                      total ms   launches   mean ms")
for k, (ns, n) in sorted(per.items(), key=lambda kv: -kv[1][0])[:24]:
    print(f"  {k:24s} {ns / 1e6:9.3f} {n:9d} {ns / n / 1e6:9.3f}")
