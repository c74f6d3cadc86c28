"""Config 5 measurement: streaming replay decode of a REMPI_DIR.

Writes R synthetic rank files (the bench workload at E events/rank, CDC-encoded on the GPU)
into a directory, then decodes the whole directory with rempi_amd.replay (file read ->
pinned host buffer -> H2D -> decode kernels -> D2H of the tables -> per-rank table dumps),
and prints one JSON line.  Under torchrun each process takes the ranks r with
r * WORLD_SIZE // R == RANK (contiguous blocks, as rempi_amd/shard.py); no collective.

    python tools/replay_bench.py --ranks 4096 --events 100000 --dir /tmp/rempi_dir
"""
import argparse
import hashlib
import json
import os
import shutil
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from rempi_amd import cdcx, replay  # noqa: E402


def write_dir(d, ranks, world, events, batch, device, perm_sha=None):
    """Encode the ranks' synthetic traces on the GPU into d/rank_<r>.rempi.  perm_sha (a dict):
    also decode every batch right there (cdcx_decode_batch_device) and keep the SHA-256 of each
    rank's permutated indices, for the check of what the replay pipeline delivers later."""
    ctx = cdcx.Context(device=device)
    s = cdcx.stream_create()
    p = cdcx.default_gen_params(world_size=world, events_per_rank=events)
    total = 0
    try:
        for b0 in range(ranks.start, ranks.stop, batch):
            n = min(batch, ranks.stop - b0)
            d_rec, rec_off = ctx.generate_device(p, b0, n, stream=s)
            d_out, off, ln = ctx.encode_batch_device(d_rec, rec_off, stream=s)
            cdcx.stream_sync(s)
            img = cdcx.d2h(d_out, int(off[-1] + ln[-1]))
            for i in range(n):
                with open(os.path.join(d, f"rank_{b0 + i}.rempi"), "wb") as f:
                    f.write(img[off[i]:off[i] + ln[i]].tobytes())
            total += int(rec_off[-1])
            if perm_sha is not None:
                _, _, d_perm = ctx.decode_batch_device(d_out, off, ln, stream=s)
                _, po = ctx.decode_rank_offsets(n)
                perm = cdcx.d2h(d_perm, int(po[-1]) * 4, np.int32)
                for i in range(n):
                    perm_sha[b0 + i] = hashlib.sha256(memoryview(np.ascontiguousarray(perm[po[i]:po[i + 1]]))).hexdigest()
    finally:
        ctx.close()
    return total


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=4096)
    ap.add_argument("--events", type=int, default=100_000)
    ap.add_argument("--dir", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "rempi_dir"))
    ap.add_argument("--streams", type=int, default=4)
    ap.add_argument("--batch-mb", type=int, default=256)
    ap.add_argument("--gen-batch", type=int, default=64)
    ap.add_argument("--repeat", type=int, default=2, help="decode passes (the first warms up)")
    ap.add_argument("--keep", action="store_true")
    ap.add_argument("--verify", type=int, default=1,
                    help="after the timed passes, one more pass that hashes every file's delivered permutated indices "
                         "against the encoder-side decode of the same file")
    ap.add_argument("--py-sink", action="store_true", help="hand every dump to a Python sink (bytes copy)")
    ap.add_argument("--tables", action="store_true",
                    help="deliver flat tables per chunk (cdcx_replay_decode_tables) instead of int64 dumps")
    a = ap.parse_args()
    ws, rank = int(os.environ.get("WORLD_SIZE", 1)), int(os.environ.get("RANK", 0))
    dev = int(os.environ.get("LOCAL_RANK", 0))
    lo = next(r for r in range(a.ranks + 1) if r == a.ranks or r * ws // a.ranks == rank)
    hi = next(r for r in range(lo, a.ranks + 1) if r == a.ranks or r * ws // a.ranks > rank)
    d = f"{a.dir}_{rank}"
    os.makedirs(d, exist_ok=True)
    t0 = time.perf_counter()
    perm_sha = {} if a.verify else None
    records = write_dir(d, range(lo, hi), a.ranks, a.events, a.gen_batch, dev, perm_sha)
    t_write = time.perf_counter() - t0
    n_dumped = [0]

    def sink(r, data):  # a consumer that takes each rank's tables (a bytes copy)
        n_dumped[0] += 1

    n_tables = [0]

    def table_sink(r, n_chunks, chunks):  # a consumer that walks the descriptors it is handed
        for k in range(n_chunks):
            n_tables[0] += chunks[k].n_tables

    st = None
    for _ in range(max(a.repeat, 1)):
        n_dumped[0] = 0
        n_tables[0] = 0
        if a.tables:
            st, _ = replay.decode_dir_tables(d, a.streams, a.batch_mb << 20, 0, dev, table_sink, convert=False)
        else:
            st, _ = replay.decode_dir(d, a.streams, a.batch_mb << 20, 0, dev, sink if a.py_sink else None)
    # Untimed: every file's permutated indices as the pipeline delivers them, hashed and compared
    # with the encoder-side decode of the same file (write_dir).
    verify = None
    if a.verify:
        seen, bad = set(), []

        def check_sink(r, n_chunks, chunks):
            h = hashlib.sha256()
            for k in range(n_chunks):
                for q in range(chunks[k].n_tables):
                    t = chunks[k].tables[q]
                    if t.count:
                        h.update(memoryview(np.ctypeslib.as_array(t.perm, shape=(t.count,))))
            seen.add(r)
            if h.hexdigest() != perm_sha.get(r):
                bad.append(r)

        replay.decode_dir_tables(d, a.streams, a.batch_mb << 20, 0, dev, check_sink, convert=False)
        missing = sorted(set(perm_sha) - seen)
        verify = {"files_checked": len(seen), "files_failed": len(bad) + len(missing), "failed_ranks": (bad + missing)[:16],
                  "how": "SHA-256 of each file's permutated indices from the table sink against "
                         "cdcx_decode_batch_device of the same file right after it was encoded"}
    if not a.keep:
        shutil.rmtree(d, ignore_errors=True)
    out = {
        "what": "config 5: streaming replay decode of REMPI_DIR rank files (read -> pinned -> H2D -> decode -> D2H "
                "tables -> " + ("flat tables per chunk handed to the sink in place" if a.tables else "per-rank dumps")
                + "), page cache warm",
        "mode": "tables" if a.tables else "dumps", "tables_seen": n_tables[0],
        "ranks": hi - lo, "world": a.ranks, "events_per_rank": a.events, "streams": a.streams,
        "records_written": records, "write_s": round(t_write, 2),
        "files": st["files"], "file_gb": round(st["file_bytes"] / 1e9, 3), "records_decoded": st["records"],
        "chunks": st["chunks"], "units": st["units"], "batches": st["batches"], "seconds": round(st["seconds"], 3),
        "record_gbps": round(32 * st["records"] / st["seconds"] / 1e9, 2),
        "file_gbps": round(st["file_bytes"] / st["seconds"] / 1e9, 2),
        "dump_gb": round(st["dump_bytes"] / 1e9, 3), "py_sink_dumps": n_dumped[0],
        "thread_s": {k: round(st[k], 3) for k in ("read_s", "device_s", "dump_s", "sink_s")},
        "verify": verify,
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
