"""Per-kernel table from the rocprofv3 --pmc passes of tools/pmc_all.sh: total per kernel name
over the run (all dispatches) of VALU/SALU/LDS/VMEM instructions, waves, and HBM bytes (read =
2 x FETCH_SIZE KiB, the gfx950 correction of tools/pmc_traffic.py; write = WRITE_SIZE KiB).

usage: python tools/pmc_table.py <dir> [records] [out.json]"""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("cdcx::", "")
        k = {"k_chain_grp<16>": "k_chain_grp16", "k_chain_grp<64>": "k_chain_grp64", "k_epoch<512>": "k_epoch",
             "k_dec_perm_seg<0>": "k_dec_perm_grp", "k_dec_perm_seg<1>": "k_dec_perm_seg", "k_dec_perm_seg<2>": "k_dec_perm_redo",
             "k_chain_seg<16>": "k_chain_seg"}.get(k, k)
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
recs = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
rows = []
for k, c in acc.items():
    rd, wr = 2.0 * 1024.0 * c.get("FETCH_SIZE", 0.0), 1024.0 * c.get("WRITE_SIZE", 0.0)
    rows.append((c.get("SQ_INSTS_VALU", 0.0), k, c, rd, wr))
rows.sort(reverse=True)
tv = sum(r[0] for r in rows) or 1.0
tb = sum(r[3] + r[4] for r in rows) or 1.0
print(f"{'kernel':24s} {'VALU':>10s} {'%':>6s} {'SALU':>10s} {'LDS':>9s} {'VMEM':>9s} {'waves':>8s} {'read GB':>8s} {'write GB':>8s} {'B/rec':>7s}")
out = {"records": recs, "fetch_correction": 2.0, "kernels": {}}
for v, k, c, rd, wr in rows:
    if k.startswith("k_gen") or k.startswith("__amd"):
        continue
    print(f"{k:24s} {v / 1e6:9.1f}M {100 * v / tv:6.1f} {c.get('SQ_INSTS_SALU', 0) / 1e6:9.1f}M {c.get('SQ_INSTS_LDS', 0) / 1e6:8.1f}M "
          f"{(c.get('SQ_INSTS_VMEM_RD', 0) + c.get('SQ_INSTS_VMEM_WR', 0)) / 1e6:8.1f}M {c.get('SQ_WAVES', 0):8.0f} {rd / 1e9:8.3f} {wr / 1e9:8.3f} "
          f"{(rd + wr) / recs if recs else 0:7.2f}")
    out["kernels"][k] = {"valu": v, "salu": c.get("SQ_INSTS_SALU", 0), "waves": c.get("SQ_WAVES", 0), "read_bytes": round(rd),
                         "write_bytes": round(wr), "dispatches": len(disp[k]),
                         "bytes_per_record": round((rd + wr) / recs, 3) if recs else None}
codec = [r for r in rows if not (r[1].startswith("k_gen") or r[1].startswith("__amd"))]
if recs:
    out["pipeline_bytes_per_record"] = round(sum(r[3] + r[4] for r in codec) / recs, 2)
    out["pipeline_valu_per_record"] = round(sum(r[0] for r in codec) / recs, 2)
    print(f"codec kernels: {out['pipeline_bytes_per_record']} HBM B/record, {out['pipeline_valu_per_record']} VALU wave-instructions/record")
if len(sys.argv) > 3:
    json.dump(out, open(sys.argv[3], "w"), indent=1)
