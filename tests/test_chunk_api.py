"""Per-chunk replay-side entry points (cdcx_decode_chunk, cdcx_reconstruct_chunk) and the
footer writer (cdcx_footer) against the reference-written golden files: what a drop-in
rempi_encoder_cdc::decode / write_footer replacement calls."""
import numpy as np
import pytest

import cdc_streams as S
import golden_util as G
import oracle_lib as O
import rempi_amd
from rempi_amd import cdcx

OK_NAMES = [n for n in G.names() if not G.load(n)["ref_failed"]]


def chunks_of(data: bytes):
    """-> ([payload bytes per chunk], footer offset (of the separator))"""
    out, p = [], 0
    while True:
        n = int(np.frombuffer(data[p:p + 8], np.uint64)[0])
        if n == 0:
            return out, p
        out.append(data[p + 8:p + 8 + n])
        p += 8 + n


@pytest.mark.parametrize("name", OK_NAMES)
def test_footer_matches_reference_file(name):
    """cdcx_footer needs no GPU: feed it the epoch ranks in the order format() inserts them
    (chunk by chunk, table by table) and compare with the reference file's footer bytes."""
    d = G.load(name)
    _, foot = chunks_of(d["rempi"])
    ranks = [int(x) for ch in O.parse_tables(d["tables"]) for t in ch for x in t["epoch_rank"]]
    assert cdcx.footer(ranks) == d["rempi"][foot:]


def test_footer_capacity_and_rehash_boundaries():
    import ctypes
    L = rempi_amd.lib()
    r = np.arange(40, dtype=np.int32)
    n = ctypes.c_size_t(10)
    out = np.zeros(10, np.uint8)
    rc = L.cdcx_footer(r.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), r.size,
                       out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), ctypes.byref(n))
    assert rc == 1 and n.value == 20 + 4 * 40
    for k in (0, 1, 13, 14, 29, 30, 59, 60, 127, 128, 600):
        keys = (np.arange(k, dtype=np.int64) * 7 + 3).astype(np.int32)
        f = cdcx.footer(np.concatenate([keys, keys[::-1]]))  # re-inserting changes nothing
        want = O.uset_int_order(keys)
        assert np.frombuffer(f[:16], np.uint64).tolist() == [0, k]
        np.testing.assert_array_equal(np.frombuffer(f[16:16 + 4 * k], np.int32), want)
        assert f[16 + 4 * k:] == b"\0\0\0\0"


@pytest.mark.gpu
@pytest.mark.parametrize("name", OK_NAMES)
def test_decode_chunk_golden(name):
    d = G.load(name)
    c = rempi_amd.Context(d["max_len"])
    payloads, _ = chunks_of(d["rempi"])
    want = O.parse_tables(d["tables"])
    assert len(payloads) == len(want)
    for pl, wt in zip(payloads, want):
        got = c.decode_chunk(pl)
        assert [t["set_id"] for t in got] == [t["set_id"] for t in wt]
        for g, w in zip(got, wt):
            assert g["count"] == w["count"]
            for k in ("epoch_rank", "epoch_clock", "with_previous", "matched_index", "ids", "delays", "perm"):
                np.testing.assert_array_equal(g[k], w[k], err_msg=k)
            um = dict(zip(g["unmatched_id"].tolist(), g["unmatched_count"].tolist()))  # umap[id] = count
            assert sorted(um.items()) == [tuple(x) for x in w["unmatched"].tolist()]
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["kat", "multichunk_small_max", "groups_heavy", "unmatched_heavy", "s5000_jitter4_t2_m16"])
def test_reconstruct_chunk_golden(name):
    d = G.load(name)
    c = rempi_amd.Context(d["max_len"])
    payloads, _ = chunks_of(d["rempi"])
    bounds = S.chunk_bounds(d["rec"], d["max_len"])
    assert len(bounds) == len(payloads)
    for pl, (a, b) in zip(payloads, bounds):
        recs = d["rec"][a:b]
        keys = O.sorted_keys(recs, 1 << 40)
        got = c.reconstruct_chunk(pl, keys)
        np.testing.assert_array_equal(got, S.expected_table_streams(recs, 1 << 40))
    c.close()


@pytest.mark.gpu
def test_decode_chunk_rejects_damage():
    d = G.load("kat")
    c = rempi_amd.Context(131072)
    pl = chunks_of(d["rempi"])[0][0]
    for bad in (pl[:-8], pl + b"\0" * 8, pl[:8] + b"\xff" * 8 + pl[16:]):
        with pytest.raises(cdcx.CdcxError) as e:
            c.decode_chunk(bad)
        assert e.value.code == 4
    assert c.decode_chunk(pl)[0]["count"] == 10
    c.close()
