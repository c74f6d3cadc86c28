"""REMPI_GZIP=1 stage: host zlib over the GPU's CDC chunks must give the
reference's own REMPI_GZIP=1 files byte for byte (fixtures written by the reference encoder,
tests/golden/make_gzip_golden.py), and gzip contexts must encode / decode them."""
import numpy as np
import pytest

import golden_util as G
import oracle_lib as O
import rempi_amd
from rempi_amd import cdcx

NAMES = G.gzip_names()


def test_fixtures_present():
    assert len(NAMES) >= 5


@pytest.mark.parametrize("name", NAMES)
def test_gzip_stage_matches_reference(name):
    d = G.load_gzip(name)
    assert cdcx.gzip_file(d["rempi"]) == d["rempi_gz"]
    assert cdcx.gunzip_file(d["rempi_gz"]) == d["rempi"]


def test_gunzip_rejects_corrupt_chunk():
    d = G.load_gzip("gzip_kat")
    bad = bytearray(d["rempi_gz"])
    bad[20] ^= 0xFF
    with pytest.raises(cdcx.CdcxError) as e:
        cdcx.gunzip_file(bytes(bad))
    assert e.value.code == 4
    with pytest.raises(cdcx.CdcxError):
        cdcx.gunzip_file(d["rempi_gz"][:-30])


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gzip_context_encode_decode(name):
    d = G.load_gzip(name)
    c = rempi_amd.Context(d["max_len"], gzip=1)
    assert c.encode_stream(d["rec"]) == d["rempi_gz"]
    assert c.decode_stream(d["rempi_gz"]) == d["tables"]
    keys = O.sorted_keys(d["rec"], d["max_len"])
    np.testing.assert_array_equal(c.reconstruct_stream(d["rempi_gz"], keys), O.reconstruct(d["rempi"], keys))
    c.close()


@pytest.mark.gpu
def test_gzip_context_rejects_device_batches():
    c = rempi_amd.Context(131072, gzip=1)
    p = rempi_amd.default_gen_params(world_size=16, events_per_rank=2000)
    d_rec, rec_off = c.generate_device(p, 0, 2)
    with pytest.raises(cdcx.CdcxError) as e:
        c.encode_batch_device(d_rec, rec_off)
    assert e.value.code == 1
    c.close()
