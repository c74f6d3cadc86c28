"""Config 1 of BASELINE.json (plumbing): the streams of `rempi_test_units matching` on 4 ranks
(emulated by tests/golden/make_config1_golden.py, encoded and decoded by the reference).  The 4
ranks are encoded on the GPU, written as a REMPI_DIR and replayed through the streaming decode;
bytes and tables must be the reference's."""
import numpy as np
import pytest

import cdc_streams as S
import golden_util as G
import oracle_lib as O
import rempi_amd
from rempi_amd import replay

RANKS = ["config1_matching_r0_seed1", "config1_matching_r1", "config1_matching_r2", "config1_matching_r3"]


def test_config1_streams_have_the_shape_of_the_matching_test():
    d = G.load(RANKS[0])
    rec = d["rec"]
    m = rec[rec[:, 2] == 1]
    assert m.shape[0] == 8 * 3 * 4                        # 8 matching functions x 3 senders x NUM_TEST_MSG 4
    assert sorted(set(m[:, 7])) == list(range(8))         # one matching set per function
    assert set(m[:, 3]) == {1, 2, 3}
    for s in (1, 2, 3):                                   # per-sender clocks strictly increase
        assert (np.diff(m[m[:, 3] == s][:, 6]) > 0).all()
    assert (m[m[:, 7] == 3][:, 4].reshape(-1, 3) == [1, 1, 0]).all()  # Testall: groups of num_sender
    assert (rec[rec[:, 7] >= 4][:, 2] == 1).all()         # Wait*: no unmatched polls
    for r in RANKS[1:]:
        assert G.load(r)["rec"].shape[0] == 0 and len(G.load(r)["rempi"]) == 20
    assert O.encode(rec, d["max_len"])[0] == d["rempi"]


@pytest.mark.gpu
def test_config1_four_ranks_encode_and_replay(tmp_path):
    c = rempi_amd.Context(131072)
    for r, name in enumerate(RANKS):
        d = G.load(name)
        got = c.encode_stream(d["rec"])
        assert got == d["rempi"], name
        (tmp_path / f"rank_{r}.rempi").write_bytes(got)
        keys = O.sorted_keys(d["rec"], d["max_len"])
        np.testing.assert_array_equal(c.reconstruct_stream(got, keys), S.expected_table_streams(d["rec"], d["max_len"]))
    c.close()
    got = {}
    st, ranks = replay.decode_dir(str(tmp_path), streams=2, sink=lambda r, b: got.__setitem__(r, b))
    assert ranks == [0, 1, 2, 3] and st["files"] == 4
    for r, name in enumerate(RANKS):
        assert got[r] == G.load(name)["tables"], name
