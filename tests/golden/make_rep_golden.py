"""Regenerate tests/golden/rep_*.npz from the REFERENCE rep encoder (REMPI_ENCODE=7,
rempi_encoder_rep; oracle/_ref/ref_cdc built from /root/reference by `make -C oracle ref`):

    python tests/golden/make_rep_golden.py

Each fixture holds `rec`, `max_len`, `rempi_rep` (the reference's REMPI_ENCODE=7 file for the
events) and `tables` (the reference CDC decoder's table dump of that file; rempi_encoder_rep
inherits decode() from rempi_encoder_cdc).  Data only; no reference source is stored.
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
    yield "only_unmatched", S.gen_stream(3, 500, n_sets=3, n_senders=4, jitter=0, p_unmatched=1.0), 131072
    yield "multichunk_small_max", S.gen_stream(7, 3000, n_sets=4, n_senders=16, jitter=8), 64
    yield "groups_heavy", S.gen_stream(9, 4000, n_sets=2, n_senders=300, jitter=32, p_group=0.6), 512
    import rempi_amd as ra

    p = ra.default_gen_params(world_size=64, events_per_rank=30000)
    yield "synthetic_w64_r5_30k", ra.generate_host(p, 5), 4096


def main():
    if not O.have_ref():
        sys.exit("oracle/_ref/ref_cdc missing: make -C oracle ref")
    for name, rec, mx in cases():
        rep, _ = O.ref_encode(rec, mx, rep=True)
        tables, _ = O.ref_decode(rep)
        np.savez_compressed(os.path.join(HERE, f"rep_{name}.npz"), rec=rec, max_len=np.int64(mx),
                            rempi_rep=np.frombuffer(rep, np.uint8), tables=np.frombuffer(tables, np.uint8))
        print(f"rep_{name}: {len(rec)} records, rep file {len(rep)} B")


if __name__ == "__main__":
    main()
