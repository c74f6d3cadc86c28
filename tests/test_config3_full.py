"""Config 3 at full size, pinned to the reference: 10 M-event ranks (77 chunks each) of the
1024-rank bench workload run through the device batch path in the bench's own layout (4
lanes x 24 rank traces on 4 HIP streams, one context and host thread per lane) and are
compared with tests/golden/config3_full.json -- SHA-256 of the file the REFERENCE encoder
wrote for the same trace, of the REFERENCE decoder's permutation and table dump, and of
the expected reconstructed records (tests/golden/make_config3_golden.py).  Every rank of
every lane is also checked by the device-side round trip."""
import hashlib
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import rempi_amd  # noqa: E402
from rempi_amd import cdcx, shard  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fixture():
    with open(bench.FIXTURE) as f:
        fx = json.load(f)
    return fx, {int(k): v for k, v in fx["ranks"].items()}


def _params(fx):
    g = fx["generator"]
    return rempi_amd.default_gen_params(world_size=g["world_size"], senders=g["senders"], sets=g["sets"],
                                        jitter=g["jitter"], events_per_rank=g["events_per_rank"], seed_salt=g["seed_salt"])


def test_fixture_pins_full_size_ranks(fixture):
    fx, ranks = fixture
    assert fx["generator"]["events_per_rank"] == 10_000_000 and fx["max_len"] == 131072
    assert {0, 95, 1023} <= set(ranks) and len(ranks) >= 4
    assert all(v["chunks"] == 77 for v in ranks.values())


def test_bench_layout_matches_reference_hashes(fixture):
    fx, ranks = fixture
    p = _params(fx)
    lanes = [bench.Lane(fx["max_len"], 0) for _ in range(4)]
    try:
        # batch 1: ranks 0..95 as the bench lays them out at 96 resident traces; batch 2: the job's last 24 ranks
        for first, count, want in ((0, 96, {0, 47, 71, 95}), (1000, 24, {1023})):
            sizes = shard.lane_sizes(count, 4)
            at = first
            for ln, n in zip(lanes, sizes):
                ln.load(p, at, n)
                at += n
            bench.run_lanes(lanes, bench.Lane.step, 2)  # a second step reuses every scratch buffer
            seen = set()
            for ln in lanes:
                v = bench.verify_lane(ln, ranks)
                assert v["dec_fail"] == 0 and v["enc_fail"] == 0, v["notes"]
                assert v["dec_ranks"] == ln.n
                seen |= {r for r in ranks if ln.first <= r < ln.first + ln.n}
            assert seen == want & set(ranks)
        # the checker is not vacuous: damage one decoded record on the device
        ln = lanes[0]
        d_recs = ln.last[3]
        one = np.array([12345], np.int32)
        assert cdcx.hip().hipMemcpy(d_recs + 32 * 777 + 12, one.ctypes.data, 4, 1) == 0
        assert ln.ctx.verify_roundtrip_device(ln.d_rec, stream=ln.stream) == 1
    finally:
        for ln in lanes:
            ln.close()


def test_table_dump_of_a_full_rank_matches_reference_decoder(fixture):
    """cdcx_decode_stream of one 147 MB rank file (77 chunks, 308 tables): the int64 table dump
    hashes to the reference decode()'s dump of the reference's own file."""
    fx, ranks = fixture
    r = 1023
    c = rempi_amd.Context(fx["max_len"])
    d_rec, rec_off = c.generate_device(_params(fx), r, 1)
    d_out, off, ln = c.encode_batch_device(d_rec, rec_off)
    data = cdcx.d2h(d_out + int(off[0]), int(ln[0])).tobytes()
    assert hashlib.sha256(data).hexdigest() == ranks[r]["file_sha256"]
    dump = c.decode_stream(data)
    assert len(dump) == ranks[r]["tables_len"]
    assert hashlib.sha256(dump).hexdigest() == ranks[r]["tables_sha256"]
    c.close()
