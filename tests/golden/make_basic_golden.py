"""Regenerate tests/golden/basic_*.npz from the REFERENCE encoders (oracle/_ref/ref_cdc, built
from /root/reference by `make -C oracle ref`).  Run in the development container:

    python tests/golden/make_basic_golden.py

Each fixture holds `rec` (n x 8 int32 canonical input), `max_len`, `basic` (the file the
reference REMPI_ENCODE=0 encoder writes for it: rempi_encoder_basic, `ref_cdc encode_basic`)
and `rempi` (the file the reference CDC encoder writes for the same events), and `basic_gz`
(the REMPI_GZIP=1 basic file: zlib chunk payloads).  They pin the
basic -> CDC transcoder (cdcx_transcode_basic): reading the reference's own basic files must
give the reference's own CDC files.  Data only; no reference source is stored.
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
    yield "groups_heavy", S.gen_stream(9, 2000, n_sets=3, n_senders=12, jitter=4, p_group=0.6), 64
    yield "unmatched_heavy", S.gen_stream(8, 2000, n_sets=2, n_senders=8, jitter=4, p_unmatched=0.9), 100
    import rempi_amd as ra

    p = ra.default_gen_params(world_size=64, events_per_rank=30000)
    yield "synthetic_w64_r3_30k", ra.generate_host(p, 3), 131072


def main():
    if not O.have_ref():
        sys.exit("oracle/_ref/ref_cdc missing: make -C oracle ref")
    for name, rec, mx in cases():
        basic = O.ref_encode_basic(rec, mx)
        basic_gz = O.ref_encode_basic(rec, mx, gzip=True)
        rempi, _ = O.ref_encode(rec, mx)
        assert np.array_equal(O.parse_basic(basic), rec), name
        np.savez_compressed(os.path.join(HERE, f"basic_{name}.npz"), rec=rec, max_len=np.int64(mx),
                            basic=np.frombuffer(basic, np.uint8), basic_gz=np.frombuffer(basic_gz, np.uint8),
                            rempi=np.frombuffer(rempi, np.uint8))
        print(f"basic_{name}: {len(rec)} records, basic {len(basic)} B, cdc {len(rempi)} B")


if __name__ == "__main__":
    main()
