"""Fixtures for the footer's matching-set-id map (write_footer / read_footer,
rempi_encoder_cdc.cpp:2015-2126), written by the REFERENCE (oracle/_ref/ref_cdc): the harness
registers the map through the reference's own rempi_reqmg_set_matching_set_id_map before
close_record_file, and dumps what rempi_reqmg_get_matching_set_id_map returns after the
reference's read_footer has read the file back.  Run in the development container:

    python tests/golden/make_footer_golden.py

Each footer_*.npz holds: rec, max_len, map_ids / map_sets (registration order, duplicates
included), rempi (the reference's file) and readback (int64: L, msg ids, set ids as the
reference returns them after read_footer).  Data only."""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import cdc_streams as S  # noqa: E402
import oracle_lib as O  # noqa: E402


def cases():
    rng = np.random.default_rng(77)
    kat = S.kat_stream()
    yield "footer_map_small", kat, 131072, [7, 3, 12], [1, 0, 2]
    yield "footer_map_overwrite", kat, 131072, [5, 9, 5, 1 << 40, 9], [1, 2, 3, 4, 5]
    # past the 13 -> 29 and 29 -> 59 bucket growths of libstdc++'s hash table
    ids = [int(x) for x in rng.choice(1 << 20, size=40, replace=False)]
    yield "footer_map_rehash", S.gen_stream(3, 800, n_sets=3, n_senders=9, jitter=4), 64, ids, [int(x) for x in rng.integers(0, 8, 40)]
    # message ids as rempi_mpi_get_msg_id builds them: communicator id in the high word, tag in the low
    ids = [(c << 32) | t for c in (0, 1, 5) for t in (0, 1, 77, 32767)]
    yield "footer_map_comm_tag", S.gen_stream(4, 300, n_sets=2, n_senders=5, jitter=8), 131072, ids, list(range(len(ids)))


def main():
    for name, rec, mx, ids, sets in cases():
        with tempfile.TemporaryDirectory() as d:
            inp, outp, mapf, back = (os.path.join(d, n) for n in ("in.rec", "out.rempi", "map.bin", "back.bin"))
            np.ascontiguousarray(rec, np.int32).tofile(inp)
            np.array([[i, s] for i, s in zip(ids, sets)], np.int64).tofile(mapf)
            subprocess.run([O.REF_BIN, "encode", inp, outp, str(mx)], check=True, capture_output=True,
                           env=dict(os.environ, REF_CDC_IDMAP=mapf))
            subprocess.run([O.REF_BIN, "footer", outp, back], check=True, capture_output=True)
            rempi = np.fromfile(outp, np.uint8)
            readback = np.fromfile(back, np.int64)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), rec=np.asarray(rec, np.int32), max_len=np.int64(mx),
                            map_ids=np.array(ids, np.uint64), map_sets=np.array(sets, np.int32), rempi=rempi,
                            readback=readback)
        print(name, rempi.size, "bytes, map entries read back:", int(readback[0]))


if __name__ == "__main__":
    main()
