"""REMPI_GZIP=1 with chunk payloads beyond ZLIB_CHUNK (1 MiB), against the reference's own
files (tests/golden/gzip_big.json, made by make_gzip_big_golden.py): the reference hands
zlib's input and output over in 1 MiB pieces (rempi_compression_util.cpp:261-283, :347-376);
the stage here makes one call per chunk and must still give the reference's bytes."""
import hashlib
import json
import os

import numpy as np
import pytest

import golden_util as G
import oracle_lib as O
import rempi_amd
from rempi_amd import cdcx

with open(os.path.join(G.GOLDEN, "gzip_big.json")) as f:
    BIG = json.load(f)


def sha(b):
    return hashlib.sha256(b).hexdigest()


def trace(c):
    p = rempi_amd.default_gen_params(world_size=c["world_size"], events_per_rank=c["events_per_rank"])
    return rempi_amd.generate_host(p, c["rank"])


@pytest.mark.parametrize("name", sorted(BIG))
def test_host_zlib_stage_matches_reference_files(name):
    """No GPU: CPU-oracle plain file -> cdcx_gzip_file -> the reference's REMPI_GZIP=1 bytes, and
    back.  Also pins the CPU oracle at a full default-REMPI_MAX chunk."""
    c = BIG[name]
    assert c["first_chunk_payload"] > (1 << 20)
    plain, _ = O.encode(trace(c), c["max_len"])
    assert len(plain) == c["rempi_len"] and sha(plain) == c["rempi_sha256"]
    gz = cdcx.gzip_file(plain)
    assert len(gz) == c["rempi_gz_len"] and sha(gz) == c["rempi_gz_sha256"]
    assert cdcx.gunzip_file(gz) == plain
    with pytest.raises(cdcx.CdcxError):  # bytes after a chunk's zlib stream are damage, not padding
        first = int(np.frombuffer(gz[:8], np.uint64)[0])
        cdcx.gunzip_file(np.uint64(first + 8).tobytes() + gz[8:8 + first] + b"\0" * 8 + gz[8 + first:])
    tables = O.decode(plain)
    assert len(tables) == c["tables_len"] and sha(tables) == c["tables_sha256"]


def test_big_case_crosses_one_mib_on_both_sides():
    assert BIG["max_1m"]["first_chunk_zlib"] > (1 << 20)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(BIG))
def test_gzip_context_matches_reference_files(name):
    c = BIG[name]
    ctx = rempi_amd.Context(c["max_len"], gzip=1)
    gz = ctx.encode_stream(trace(c))
    assert len(gz) == c["rempi_gz_len"] and sha(gz) == c["rempi_gz_sha256"]
    tables = ctx.decode_stream(gz)
    assert len(tables) == c["tables_len"] and sha(tables) == c["tables_sha256"]
    ctx.close()
