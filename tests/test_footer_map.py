"""The footer's matching-set-id map (write_footer / read_footer, rempi_encoder_cdc.cpp:2015-2126)
against files the reference wrote with a map registered through its own
rempi_reqmg_set_matching_set_id_map (tests/golden/footer_*.npz): the footer writer and reader of
the C ABI on the host, the host-buffer encoder of a context with a registered map, and the
replay pipeline's footer sink."""
import os

import numpy as np
import pytest

import golden_util as G
import oracle_lib as O
import rempi_amd
from rempi_amd import cdcx

NAMES = G.footer_names()


def footer_of(data: bytes) -> bytes:
    p = 0
    while True:
        n = int(np.frombuffer(data[p:p + 8], np.uint64)[0])
        if n == 0:
            return data[p:]
        p += 8 + n


def epoch_ranks_in_insertion_order(data: bytes):
    """format() adds every table's epoch ranks to all_epoch_rank_uset, chunk by chunk, table by table."""
    return [int(x) for chunk in O.parse_tables(O.decode(data)) for t in chunk for x in t["epoch_rank"]]


def test_fixtures_present():
    assert len(NAMES) >= 4


@pytest.mark.parametrize("name", NAMES)
def test_footer_writer_matches_reference(name):
    d = G.load_footer(name)
    got = cdcx.footer(epoch_ranks_in_insertion_order(d["rempi"]), d["map_ids"], d["map_sets"])
    assert got == footer_of(d["rempi"])


@pytest.mark.parametrize("name", NAMES)
def test_footer_reader_matches_reference(name):
    d = G.load_footer(name)
    f = cdcx.read_footer(d["rempi"])
    # the file holds the map in the writer's hash order; after read_footer has registered the
    # entries in that order, the reference's map iterates as `readback`
    L = int(d["readback"][0])
    assert f["msg_ids"].size == L == len(set(int(x) for x in d["map_ids"]))
    again = cdcx.footer([], f["msg_ids"], f["set_ids"])  # (hash order after registering in file order)
    g = cdcx.read_footer(np.zeros(8, np.uint8).tobytes()[:0] + again)
    np.testing.assert_array_equal(g["msg_ids"].astype(np.int64), d["readback"][1:1 + L])
    np.testing.assert_array_equal(g["set_ids"].astype(np.int64), d["readback"][1 + L:])
    # the last registration of an id wins
    want = {}
    for i, s in zip(d["map_ids"], d["map_sets"]):
        want[int(i)] = int(s)
    assert {int(i): int(s) for i, s in zip(f["msg_ids"], f["set_ids"])} == want
    np.testing.assert_array_equal(np.sort(f["ranks"]), np.unique(epoch_ranks_in_insertion_order(d["rempi"])))


def test_footer_reader_rejects_damage():
    d = G.load_footer(NAMES[0])
    data = d["rempi"]
    for cut in (1, 4, 11, len(footer_of(data)) - 9):
        with pytest.raises(cdcx.CdcxError) as e:
            cdcx.read_footer(data[:-cut])
        assert e.value.code == 4
    with pytest.raises(cdcx.CdcxError):
        cdcx.read_footer(data[:24])  # no separator


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_encode_stream_with_map_matches_reference(name):
    d = G.load_footer(name)
    c = rempi_amd.Context(d["max_len"])
    c.set_matching_set_id_map(d["map_ids"], d["map_sets"])
    assert c.encode_stream(d["rec"]) == d["rempi"]
    c.set_matching_set_id_map()  # forget it: the plain footer again
    plain = c.encode_stream(d["rec"])
    assert plain == O.encode(d["rec"], d["max_len"])[0]
    # decoding ignores the map (it is the replay engine's input, not table data)
    assert c.decode_stream(d["rempi"]) == O.decode(plain)
    c.close()


@pytest.mark.gpu
def test_replay_delivers_footers(tmp_path):
    from rempi_amd import replay

    want = {}
    for r, name in enumerate(NAMES):
        d = G.load_footer(name)
        with open(os.path.join(tmp_path, f"rank_{r}.rempi"), "wb") as f:
            f.write(d["rempi"])
        want[r] = cdcx.read_footer(d["rempi"])
    got, tables = {}, {}
    replay.decode_dir_tables(str(tmp_path), streams=2, sink=lambda r, chunks: tables.__setitem__(r, len(chunks)),
                             footer_sink=lambda r, f: got.__setitem__(r, f))
    assert sorted(got) == sorted(want) == sorted(tables)
    for r in want:
        for k in ("ranks", "msg_ids", "set_ids"):
            np.testing.assert_array_equal(got[r][k], want[r][k])
        assert want[r]["msg_ids"].size > 0
