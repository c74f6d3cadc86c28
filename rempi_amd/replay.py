"""Replay-side streaming decode of a REMPI_DIR (the benchmark's config 5).

In the reference every replaying rank process runs progress_decoding
(rempi_encoder_cdc.cpp:851-930): read_record_file (:933-978) -> decode (:1016-1299) ->
cdc_prepare_decode_indices (:1301-1386) over its own REMPI_DIR/rank_<r>.rempi.  Here one
process decodes many rank files per GPU through cdcx_replay_decode_files: batches of files
are read into pinned host memory, copied to the device, decoded by the HIP kernels of
decode.hip, and their tables copied back, with one host thread and HIP stream per context
so that reads, copies and kernels of different batches overlap.

    python -m rempi_amd.replay REMPI_DIR [--streams 4] [--batch-mb 256] [--gzip]
                               [--out DIR] [--ranks 0:4096]

Writes, with --out, DIR/rank_<r>.tables: the int64 table dump of cdcx_decode_stream
(oracle/tables_format.md).  Prints one JSON line of totals.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys

from . import cdcx

_RANK_FILE = re.compile(r"^rank_(\d+)\.rempi$")


def rank_files(rempi_dir: str, ranks: range | None = None) -> list[tuple[int, str]]:
    """(rank, path) of every rank_<r>.rempi under rempi_dir, by rank
    (the naming of rempi_recorder_cdc::init, rempi_recorder_cdc.cpp:135)."""
    out = []
    for name in os.listdir(rempi_dir):
        m = _RANK_FILE.match(name)
        if m and (ranks is None or int(m.group(1)) in ranks):
            out.append((int(m.group(1)), os.path.join(rempi_dir, name)))
    return sorted(out)


def decode_dir(rempi_dir: str, streams: int = 4, batch_bytes: int = 256 << 20, gzip: int = 0, device: int = 0,
               sink=None, ranks: range | None = None, max_event_length: int = 131072):
    """Decode every rank file of rempi_dir.  sink(rank, dump_bytes) gets each rank's tables.
    -> (stats dict, [rank, ...] in file-index order)."""
    files = rank_files(rempi_dir, ranks)
    ctxs = [cdcx.Context(max_event_length=max_event_length, device=device, gzip=gzip) for _ in range(max(streams, 1))]
    try:
        fwd = None if sink is None else (lambda i, data: sink(files[i][0], data))
        st = cdcx.replay_decode_files(ctxs, [p for _, p in files], fwd, batch_bytes)
    finally:
        for c in ctxs:
            c.close()
    return st, [r for r, _ in files]


def decode_dir_tables(rempi_dir: str, streams: int = 4, batch_bytes: int = 256 << 20, gzip: int = 0, device: int = 0,
                      sink=None, ranks: range | None = None, max_event_length: int = 131072, convert: bool = True,
                      devices=None, footer_sink=None):
    """Like decode_dir, but sink(rank, chunks) gets the flat tables of every chunk (what the
    reference's replay engine consumes) instead of an int64 dump.  `devices`: one device ordinal
    per context (contexts of one call may sit on different GPUs).  footer_sink(rank, footer) gets
    every file's footer (global predecessor ranks, matching-set-id map) before its tables."""
    files = rank_files(rempi_dir, ranks)
    devs = list(devices) if devices else [device] * max(streams, 1)
    ctxs = [cdcx.Context(max_event_length=max_event_length, device=d, gzip=gzip) for d in devs]
    try:
        fwd = None
        if sink is not None:
            fwd = (lambda i, *rest: sink(files[i][0], *rest))
        ffwd = None if footer_sink is None else (lambda i, footer: footer_sink(files[i][0], footer))
        st = cdcx.replay_decode_tables(ctxs, [p for _, p in files], fwd, batch_bytes, convert, ffwd)
    finally:
        for c in ctxs:
            c.close()
    return st, [r for r, _ in files]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("rempi_dir")
    ap.add_argument("--streams", type=int, default=4, help="contexts (host threads + HIP streams)")
    ap.add_argument("--batch-mb", type=int, default=256, help="rank-file bytes per device batch")
    ap.add_argument("--gzip", action="store_true", help="REMPI_GZIP=1 files (inflated on the host)")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--out", help="write rank_<r>.tables dumps here")
    ap.add_argument("--ranks", help="a:b, only ranks in [a, b)")
    a = ap.parse_args(argv)
    ranks = None
    if a.ranks:
        lo, hi = (int(x) for x in a.ranks.split(":"))
        ranks = range(lo, hi)
    sink = None
    if a.out:
        os.makedirs(a.out, exist_ok=True)

        def sink(rank, data):
            with open(os.path.join(a.out, f"rank_{rank}.tables"), "wb") as f:
                f.write(data)

    st, _ = decode_dir(a.rempi_dir, a.streams, a.batch_mb << 20, int(a.gzip), a.device, sink, ranks)
    st["record_gbps"] = 32 * st["records"] / max(st["seconds"], 1e-9) / 1e9
    st["file_gbps"] = st["file_bytes"] / max(st["seconds"], 1e-9) / 1e9
    print(json.dumps(st))
    return 0


if __name__ == "__main__":
    sys.exit(main())
