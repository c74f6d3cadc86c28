"""REMPI_GZIP=1 at chunk sizes past ZLIB_CHUNK (1 MiB; the reference's deflate / inflate loops
hand data over in 1 MiB pieces, rempi_compression_util.cpp:261-283, :347-376), pinned to the
REFERENCE (oracle/_ref/ref_cdc):

    python tests/golden/make_gzip_big_golden.py

  default_max : a 140 K-event rank at the default REMPI_MAX = 131072 -- one chunk whose plain
                payload is ~1.9 MB (inflate side crosses 1 MiB) plus a short one
  max_1m      : a 1.1 M-event rank at REMPI_MAX = 1048576 -- a ~15 MB payload whose zlib
                stream is itself several MiB (deflate side crosses 1 MiB too)

The inputs come from the host generator (cdcx_generate_host) and are not stored; the fixture
tests/golden/gzip_big.json keeps the generator parameters and the SHA-256 / length of the
reference's plain file, its REMPI_GZIP=1 file and the reference decoder's table dump.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import oracle_lib as O  # noqa: E402
import rempi_amd  # noqa: E402

CASES = {"default_max": {"world_size": 64, "events_per_rank": 140_000, "rank": 3, "max_len": 131072},
         "max_1m": {"world_size": 64, "events_per_rank": 1_100_000, "rank": 5, "max_len": 1 << 20}}


def sha(b):
    return hashlib.sha256(b).hexdigest()


def main():
    assert O.have_ref(), "oracle/_ref/ref_cdc missing: make -C oracle ref"
    out = {}
    for name, c in CASES.items():
        p = rempi_amd.default_gen_params(world_size=c["world_size"], events_per_rank=c["events_per_rank"])
        rec = rempi_amd.generate_host(p, c["rank"])
        plain, _ = O.ref_encode(rec, c["max_len"])
        gz, _ = O.ref_encode(rec, c["max_len"], gzip=True)
        tables, _ = O.ref_decode(plain)
        tables_gz, _ = O.ref_decode(gz, gzip=True)
        assert tables == tables_gz
        first_plain = int(np.frombuffer(plain[:8], np.uint64)[0])
        first_gz = int(np.frombuffer(gz[:8], np.uint64)[0])
        out[name] = dict(c, records=int(rec.shape[0]), rempi_len=len(plain), rempi_sha256=sha(plain), rempi_gz_len=len(gz),
                         rempi_gz_sha256=sha(gz), tables_len=len(tables), tables_sha256=sha(tables),
                         first_chunk_payload=first_plain, first_chunk_zlib=first_gz)
        print(name, out[name])
    with open(os.path.join(HERE, "gzip_big.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    main()
