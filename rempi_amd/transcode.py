"""Basic -> CDC transcoder: shrink existing REMPI_ENCODE=0 record files.

    python -m rempi_amd.transcode [--max-len REMPI_MAX] [--batch 16] -o OUTDIR rank_*.rempi

A basic record file (rempi_encoder_basic.cpp:205-224) holds one rank's canonical event
stream, so its CDC image (what a REMPI_ENCODE=7 recording of the same run writes) is the GPU
CDC encode of the concatenated chunks (cdcx_transcode_basic).  Output files keep the input
names (both encoders write REMPI_DIR/rank_<r>.rempi) under OUTDIR.  Files are encoded in
device batches of --batch ranks.  REMPI_GZIP=1 basic files are zlib streams; they are
inflated on the host first (--gzip).  --gzip-out writes REMPI_GZIP=1 CDC files (host zlib
stage, cdcx_gzip_file).
"""
from __future__ import annotations

import argparse
import os
import sys
import zlib

from .cdcx import Context


def inflate_basic(data: bytes) -> bytes:
    """REMPI_GZIP=1: each chunk's payload is a zlib stream (rempi_compression_util.cpp:233-387);
    returns the uncompressed basic file."""
    out, p = bytearray(), 0
    while p < len(data):
        n = int.from_bytes(data[p:p + 8], "little")
        raw = zlib.decompress(data[p + 8:p + 8 + n])
        out += len(raw).to_bytes(8, "little") + raw
        p += 8 + n
    return bytes(out)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("files", nargs="+")
    ap.add_argument("-o", "--out", required=True, help="output directory")
    ap.add_argument("--max-len", type=int, default=131072, help="REMPI_MAX of the CDC recording")
    ap.add_argument("--batch", type=int, default=16, help="rank files per device batch")
    ap.add_argument("--gzip", action="store_true", help="inputs were written with REMPI_GZIP=1")
    ap.add_argument("--gzip-out", action="store_true", help="write REMPI_GZIP=1 CDC files")
    args = ap.parse_args(argv)
    os.makedirs(args.out, exist_ok=True)
    ctx = Context(args.max_len, gzip=1 if args.gzip_out else 0)
    tin = tout = 0
    for i in range(0, len(args.files), args.batch):
        paths = args.files[i:i + args.batch]
        data = []
        for p in paths:
            with open(p, "rb") as f:
                b = f.read()
            data.append(inflate_basic(b) if args.gzip else b)
        for p, b, c in zip(paths, data, ctx.transcode_basic(data)):
            with open(os.path.join(args.out, os.path.basename(p)), "wb") as f:
                f.write(c)
            tin += len(b)
            tout += len(c)
    ctx.close()
    print(f"{len(args.files)} files: {tin} B basic -> {tout} B CDC", file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
