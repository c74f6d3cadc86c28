"""Regenerate tests/golden/gzip_*.npz from the REFERENCE CDC encoder with REMPI_GZIP=1
(oracle/_ref/ref_cdc, built from /root/reference by `make -C oracle ref`):

    python tests/golden/make_gzip_golden.py

Each fixture holds `rec`, `max_len`, `rempi` (the reference's plain CDC file), `rempi_gz` (its
REMPI_GZIP=1 file for the same events) and `tables` (the reference decoder's table dump, the
same for both files; checked here).  They pin the host zlib stage (cdcx_gzip_file,
cdcx_gunzip_file, gzip contexts).  Data only; no reference source is stored.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import cdc_streams as S  # noqa: E402
import oracle_lib as O  # noqa: E402


def cases():
    yield "kat", S.kat_stream(), 131072
    yield "empty", np.zeros((0, 8), np.int32), 131072
    yield "multichunk_small_max", S.gen_stream(7, 3000, n_sets=4, n_senders=16, jitter=8), 64
    yield "unmatched_heavy", S.gen_stream(8, 2000, n_sets=2, n_senders=8, jitter=4, p_unmatched=0.9), 100
    import rempi_amd as ra

    p = ra.default_gen_params(world_size=64, events_per_rank=30000)
    yield "synthetic_w64_r4_30k", ra.generate_host(p, 4), 4096


def main():
    if not O.have_ref():
        sys.exit("oracle/_ref/ref_cdc missing: make -C oracle ref")
    for name, rec, mx in cases():
        plain, _ = O.ref_encode(rec, mx)
        gz, _ = O.ref_encode(rec, mx, gzip=True)
        tables, _ = O.ref_decode(plain)
        tables_gz, _ = O.ref_decode(gz, gzip=True)
        assert tables == tables_gz, name
        np.savez_compressed(os.path.join(HERE, f"gzip_{name}.npz"), rec=rec, max_len=np.int64(mx),
                            rempi=np.frombuffer(plain, np.uint8), rempi_gz=np.frombuffer(gz, np.uint8),
                            tables=np.frombuffer(tables, np.uint8))
        print(f"gzip_{name}: {len(rec)} records, cdc {len(plain)} B, gzip {len(gz)} B")


if __name__ == "__main__":
    main()
