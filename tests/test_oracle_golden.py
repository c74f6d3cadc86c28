"""The CPU oracle (oracle/cdc_oracle.cpp) against the reference's own outputs.

Fixtures in tests/golden/ were produced by the reference encoder/decoder compiled from
/root/reference (tests/golden/make_golden.py); where the reference binary is present
(this container) a randomized differential run is added."""
import numpy as np
import pytest

import cdc_streams as S
import golden_util as G
import oracle_lib as O

NAMES = G.names()


@pytest.mark.parametrize("name", NAMES)
def test_oracle_encode_matches_reference(name):
    d = G.load(name)
    if d["ref_failed"]:
        with pytest.raises(O.OracleError):
            O.encode(d["rec"], d["max_len"])
        return
    data, _ = O.encode(d["rec"], d["max_len"])
    assert data == d["rempi"]


@pytest.mark.parametrize("name", [n for n in NAMES if not G.load(n)["ref_failed"]])
def test_oracle_decode_matches_reference(name):
    d = G.load(name)
    assert O.decode(d["rempi"]) == d["tables"]
    try:  # (and with the reference's unbounded walk: the same tables on well-formed files)
        O.set_reference_walk(True)
        assert O.decode(d["rempi"]) == d["tables"]
    finally:
        O.set_reference_walk(False)


def _with_delays(data: bytes, table: int, delays) -> bytes:
    """The one-chunk record file `data` with the delays of its table number `table` replaced
    (second-order prediction re-applied, rempi_compression_util.cpp:117-154)."""
    b = bytearray(data)
    q = 8
    u64 = lambda p: int(np.frombuffer(bytes(b[p:p + 8]), np.uint64)[0])  # noqa: E731
    for k in range(table + 1):
        q += 8
        esz = u64(q)
        q += 8 + 2 * esz
        for _ in range(2):  # with_previous, matched_index: {length, bytes, data}
            q += 16 + u64(q + 8)
        for _ in range(2):  # unmatched ids, counts: {bytes, data}
            q += 8 + u64(q)
        psz = u64(q)
        if k == table:
            P = psz // 8
            assert len(delays) == P
            x = np.array([0, 0] + list(delays), np.int64)
            y = (x[2:] - 2 * x[1:-1] + x[:-2]).astype(np.int32)
            b[q + 8 + 4 * P:q + 8 + 8 * P] = y.tobytes()
        q += 8 + psz
    return bytes(b)


@pytest.mark.skipif(not O.have_ref(), reason="needs the reference binary (oracle/_ref/ref_cdc)")
def test_reference_walks_through_the_list_end():
    """Delays longer than the list: the reference keeps stepping through std::list's sentinel;
    the oracle does the same with oracle_set_reference_walk(1) and refuses them by default (the
    device path's rule).  Pinned here against the reference decoder itself on the KAT file."""
    d = G.load("kat")
    tabs = O.parse_tables(d["tables"])[0]
    M, P = tabs[0]["count"], len(tabs[0]["delays"])
    for delays in ([2, -3, -3, -5, -8, -6], [M + 3, -3, -3, -5, -8, -6], [2, -3, -(2 * M + 5), -5, -8, 3 * M]):
        data = _with_delays(d["rempi"], 0, delays[:P])
        ref, _ = O.ref_decode(data)
        try:
            O.set_reference_walk(True)
            assert O.decode(data) == ref, delays
        finally:
            O.set_reference_walk(False)
        if max(abs(v) for v in delays) > M:
            with pytest.raises(O.OracleError):
                O.decode(data)
        else:
            assert O.decode(data) == ref


@pytest.mark.parametrize("name", [n for n in NAMES if not G.load(n)["ref_failed"]])
def test_oracle_records_roundtrip(name):
    d = G.load(name)
    keys = O.sorted_keys(d["rec"], d["max_len"])
    rec = O.reconstruct(d["rempi"], keys)
    np.testing.assert_array_equal(rec, S.expected_table_streams(d["rec"], d["max_len"]))


def test_kat_values():
    """Known answers for the permutation of rempi_test_compress.cpp:104-113."""
    data, _ = O.encode(S.kat_stream(), 131072)
    assert len(data) == 280
    t = O.parse_tables(O.decode(data))[0][0]
    assert list(t["ids"]) == [0, 4, 6, 7, 8, 9]
    assert list(t["delays"]) == [2, -3, -3, -5, -8, -6]
    assert list(t["perm"]) == [7, 1, 5, 8, 2, 9, 6, 4, 0, 3]
    assert t["unmatched"].tolist() == [[0, 5], [10, 3]]


def test_decode_is_inverse_permutation():
    rng = np.random.default_rng(1)
    for _ in range(200):
        M = int(rng.integers(0, 60))
        c = rng.permutation(M).astype(np.int32)
        ids, dl = O.cdc_pairs(c)
        perm = O.decode_perm(ids.astype(np.int64), dl.astype(np.int64), M)
        np.testing.assert_array_equal(perm[c], np.arange(M))


@pytest.mark.skipif(not O.have_ref(), reason="reference binary not built here")
def test_oracle_random_differential():
    rng = np.random.default_rng(11)
    for t in range(60):
        mode = ["jitter", "jitter", "sorted", "reversed", "random"][t % 5]
        recs = S.gen_stream(int(rng.integers(1 << 30)), int(rng.integers(0, 300)), n_sets=int(rng.integers(1, 5)),
                            n_senders=int(rng.integers(1, 20)), jitter=int(rng.choice([0, 4, 32])), mode=mode,
                            p_unmatched=float(rng.choice([0.0, 0.3])), p_group=float(rng.choice([0.0, 0.3])))
        mx = int(rng.choice([2, 16, 131072]))
        try:
            ob, _ = O.encode(recs, mx)
        except O.OracleError:
            ob = None
        try:
            rb, _ = O.ref_encode(recs, mx)
        except RuntimeError:
            rb = None
        assert ob == rb
        if ob is not None:
            assert O.decode(ob) == O.ref_decode(rb)[0]
