"""Rep encoder (REMPI_ENCODE=7; rempi_encoder_rep.cpp:50-146): every
table keeps its set id, matched count and epoch line; the with_previous, matched_index,
unmatched and pair sections are written empty.  Fixtures are the reference's own rep files
(tests/golden/make_rep_golden.py); rep files decode through the CDC decoder (the class
inherits decode(), rempi_encoder.h:437-459)."""
import numpy as np
import pytest

import golden_util as G
import oracle_lib as O
import rempi_amd
from rempi_amd import cdcx

NAMES = G.rep_names()


def test_fixtures_present():
    assert len(NAMES) >= 6


@pytest.mark.parametrize("name", NAMES)
def test_oracle_rep_matches_reference(name):
    d = G.load_rep(name)
    got, _ = O.encode(d["rec"], d["max_len"], rep=True)
    assert got == d["rempi_rep"]
    assert O.decode(d["rempi_rep"]) == d["tables"]


@pytest.mark.parametrize("name", NAMES)
def test_rep_is_cdc_with_sections_emptied(name):
    """Size rule: the rep file is the CDC file minus every table's section payloads."""
    d = G.load_rep(name)
    cdc, _ = O.encode(d["rec"], d["max_len"])
    t_rep = O.parse_tables(d["tables"])
    t_cdc = O.parse_tables(O.decode(cdc))
    assert len(t_rep) == len(t_cdc)
    for a, b in zip(t_rep, t_cdc):
        assert len(a) == len(b)
        for x, y in zip(a, b):
            assert x["set_id"] == y["set_id"] and x["count"] == y["count"]
            np.testing.assert_array_equal(x["epoch_rank"], y["epoch_rank"])
            np.testing.assert_array_equal(x["epoch_clock"], y["epoch_clock"])
            for k in ("with_previous", "matched_index", "unmatched", "ids", "delays"):
                assert x[k].size == 0, k


def test_rejects_unknown_encode():
    with pytest.raises(cdcx.CdcxError):
        rempi_amd.Context(131072, encode=5)


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_rep_context_matches_reference(name):
    d = G.load_rep(name)
    c = rempi_amd.Context(d["max_len"], encode=7)
    assert c.encode_stream(d["rec"]) == d["rempi_rep"]
    assert c.decode_stream(d["rempi_rep"]) == d["tables"]
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("jitter,max_len", [(8, 131072), (64, 4096)])
def test_rep_device_batch_vs_oracle(jitter, max_len):
    c = rempi_amd.Context(max_len, encode=7)
    p = rempi_amd.default_gen_params(world_size=64, jitter=jitter, events_per_rank=80000)
    d_rec, rec_off = c.generate_device(p, 2, 3)
    d_out, off, ln = c.encode_batch_device(d_rec, rec_off)
    for r in range(3):
        want, _ = O.encode(rempi_amd.generate_host(p, 2 + r), max_len, rep=True)
        got = cdcx.d2h(d_out + int(off[r]), int(ln[r])).tobytes()
        assert got == want, r
    c.close()


@pytest.mark.gpu
def test_rep_then_cdc_context_reuse():
    """A rep context and a CDC context on one device do not share state."""
    rec = rempi_amd.generate_host(rempi_amd.default_gen_params(world_size=16, events_per_rank=20000), 1)
    a = rempi_amd.Context(2048, encode=7)
    b = rempi_amd.Context(2048)
    assert a.encode_stream(rec) == O.encode(rec, 2048, rep=True)[0]
    assert b.encode_stream(rec) == O.encode(rec, 2048)[0]
    assert a.encode_stream(rec) == O.encode(rec, 2048, rep=True)[0]
    a.close()
    b.close()
