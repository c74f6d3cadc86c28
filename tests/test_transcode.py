"""Basic -> CDC transcoder: REMPI_ENCODE=0 record files, written by the
reference's own rempi_encoder_basic (fixtures from tests/golden/make_basic_golden.py), must
come out as the reference CDC encoder's files for the same events.  CPU tests pin the file
format and the claim (oracle); GPU tests run cdcx_transcode_basic."""
import numpy as np
import pytest

import cdc_streams as S
import golden_util as G
import oracle_lib as O
import rempi_amd
from rempi_amd import cdcx

NAMES = G.basic_names()


def basic_file(recs, chunk):
    """Our writer of the same format (rempi_encoder_basic.cpp:205-224), `chunk` records per chunk."""
    out = bytearray()
    for i in range(0, len(recs), chunk):
        b = np.ascontiguousarray(recs[i:i + chunk], np.int32).tobytes()
        out += np.uint64(len(b)).tobytes() + b
    return bytes(out)


def test_fixtures_present():
    assert len(NAMES) >= 6


@pytest.mark.parametrize("name", NAMES)
def test_reference_basic_file_is_the_record_stream(name):
    d = G.load_basic(name)
    np.testing.assert_array_equal(O.parse_basic(d["basic"]), d["rec"])


@pytest.mark.parametrize("name", NAMES)
def test_oracle_cdc_of_basic_records(name):
    d = G.load_basic(name)
    got, _ = O.encode(O.parse_basic(d["basic"]), d["max_len"])
    assert got == d["rempi"]


def test_basic_writer_matches_reference_framing():
    d = G.load_basic("basic_kat")
    assert basic_file(d["rec"], 1 << 30) == d["basic"]


@pytest.mark.gpu
def test_transcode_reference_files():
    by_len = {}
    for n in NAMES:
        d = G.load_basic(n)
        by_len.setdefault(d["max_len"], []).append(d)
    for mx, ds in by_len.items():
        c = rempi_amd.Context(mx)
        got = c.transcode_basic([d["basic"] for d in ds])
        for d, g in zip(ds, got):
            assert g == d["rempi"], (mx, len(d["rec"]))
        c.close()


@pytest.mark.gpu
def test_transcode_multichunk_and_batch():
    """Chunking of the basic file does not matter; a batch of files equals files one by one."""
    c = rempi_amd.Context(131072)
    rng = np.random.default_rng(11)
    recs = [S.gen_stream(int(rng.integers(1 << 30)), int(rng.integers(0, 4000)), n_sets=int(rng.integers(1, 4)),
                         n_senders=int(rng.integers(2, 40)), jitter=8) for _ in range(5)]
    files = [basic_file(r, int(rng.integers(1, 700))) for r in recs]
    got = c.transcode_basic(files)
    for r, g in zip(recs, got):
        assert g == O.encode(r, 131072)[0]
        assert c.transcode_basic([basic_file(r, 1 << 30)])[0] == g
    c.close()


@pytest.mark.gpu
def test_transcode_rejects_bad_files():
    c = rempi_amd.Context(131072)
    recs = S.gen_stream(3, 50, n_sets=1, n_senders=4, jitter=2)
    good = basic_file(recs, 1 << 30)
    recv = recs.copy()
    recv[7, 1] = 0  # an MPI_Recv event: not a CDC input
    for bad in (good[:-3], good[:5], np.uint64(33).tobytes() + b"\0" * 33, basic_file(recv, 1 << 30)):
        with pytest.raises(cdcx.CdcxError) as e:
            c.transcode_basic([bad])
        assert e.value.code == 1
    assert c.transcode_basic([good])[0] == O.encode(recs, 131072)[0]  # the context is still usable
    c.close()


@pytest.mark.parametrize("name", NAMES)
def test_gzip_basic_file_inflates_to_the_basic_file(name):
    """REMPI_GZIP=1 basic files (zlib chunk payloads, written by the reference) inflate to the
    plain basic file (rempi_amd.transcode --gzip)."""
    from rempi_amd.transcode import inflate_basic

    d = G.load_basic(name)
    assert inflate_basic(d["basic_gz"]) == d["basic"]
