"""HBM traffic per kernel from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (one pass each).

usage: python tools/pmc_traffic.py <dir with FETCH_SIZE/ and WRITE_SIZE/> <records per dispatch> <out.json>

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts the L2's memory-side read
requests at 64 B per 128 B request, so it reports half of the bytes read; it is doubled here.
The factor was checked on this pipeline's own k_tile_hist, which streams its 32 B records once:
FETCH_SIZE = 3.865 GB for 7.68 GB read (0.503).  WRITE_SIZE is taken as reported.  Both are
KiB per dispatch.  The output gives per kernel the mean traffic per dispatch and per record, so
bench.py can report `roofline.traffic` for the records one of its launches processes.
"""
import collections
import csv
import json
import os
import sys


def per_dispatch(path):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("cdcx::", "")
        acc[k].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def main():
    root, recs, out = sys.argv[1], float(sys.argv[2]), sys.argv[3]
    fetch, n = per_dispatch(os.path.join(root, "FETCH_SIZE", "run_counter_collection.csv"))
    write, _ = per_dispatch(os.path.join(root, "WRITE_SIZE", "run_counter_collection.csv"))
    res = {"records_per_dispatch": recs, "fetch_correction": 2.0, "kernels": {}}
    for k in sorted(fetch):
        rd = 2.0 * fetch[k]
        wr = write.get(k, 0.0)
        name = {"k_chain_grp<16>": "k_chain_grp16", "k_chain_grp<64>": "k_chain_grp64"}.get(k, k)
        res["kernels"][name] = {"read_bytes": round(rd), "write_bytes": round(wr), "dispatches": n[k],
                                "bytes_per_record": round((rd + wr) / recs, 3)}
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res["kernels"].items():
        print(f"{k:18s} read {v['read_bytes'] / 1e9:7.3f} GB  write {v['write_bytes'] / 1e9:7.3f} GB  "
              f"{v['bytes_per_record']:7.2f} B/record")


if __name__ == "__main__":
    main()
