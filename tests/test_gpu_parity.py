"""HIP path (libcdcx.so) against the reference's bytes/tables (golden fixtures) and the CPU
oracle on seeded random streams; batch device API against the per-rank oracle.
All through the C ABI."""
import numpy as np
import pytest

import cdc_streams as S
import golden_util as G
import oracle_lib as O
import rempi_amd
from rempi_amd import cdcx

pytestmark = pytest.mark.gpu

_ctx = {}


def ctx(max_len):
    if max_len not in _ctx:
        _ctx[max_len] = rempi_amd.Context(max_len)
    return _ctx[max_len]


def first_diff(a: bytes, b: bytes):
    n = min(len(a), len(b))
    x = np.frombuffer(a[:n], np.uint8) != np.frombuffer(b[:n], np.uint8)
    i = int(np.argmax(x)) if x.any() else n
    return f"len {len(a)} vs {len(b)}, first difference at byte {i}"


NAMES = G.names()
OK_NAMES = [n for n in NAMES if not G.load(n)["ref_failed"]]


@pytest.mark.parametrize("name", NAMES)
def test_encode_golden(name):
    d = G.load(name)
    c = ctx(d["max_len"])
    if d["ref_failed"]:
        with pytest.raises(cdcx.CdcxError) as e:
            c.encode_stream(d["rec"])
        assert e.value.code in (2, 3)
        return
    got = c.encode_stream(d["rec"])
    assert got == d["rempi"], first_diff(got, d["rempi"])


@pytest.mark.parametrize("name", OK_NAMES)
def test_decode_golden(name):
    d = G.load(name)
    got = ctx(d["max_len"]).decode_stream(d["rempi"])
    assert got == d["tables"], first_diff(got, d["tables"])


@pytest.mark.parametrize("name", OK_NAMES)
def test_records_golden(name):
    d = G.load(name)
    keys = O.sorted_keys(d["rec"], d["max_len"])
    got = ctx(d["max_len"]).reconstruct_stream(d["rempi"], keys)
    np.testing.assert_array_equal(got, S.expected_table_streams(d["rec"], d["max_len"]))


def test_random_streams_vs_oracle():
    rng = np.random.default_rng(123)
    bad = []
    for t in range(150):
        mode = ["jitter", "jitter", "sorted", "reversed", "random"][t % 5]
        recs = S.gen_stream(int(rng.integers(1 << 30)), int(rng.integers(0, 3000)), n_sets=int(rng.integers(1, 5)),
                            n_senders=int(rng.integers(1, 40)), jitter=int(rng.choice([0, 1, 4, 8, 32])), mode=mode,
                            p_unmatched=float(rng.choice([0.0, 0.2, 0.7])), p_group=float(rng.choice([0.0, 0.1, 0.5])),
                            neg_index=bool(t % 4 == 0))
        mx = int(rng.choice([1, 3, 16, 100, 131072]))
        try:
            want, _ = O.encode(recs, mx)
        except O.OracleError as e:
            with pytest.raises(cdcx.CdcxError):
                ctx(mx).encode_stream(recs)
            continue
        got = ctx(mx).encode_stream(recs)
        if got != want:
            bad.append((t, mode, recs.shape[0], mx, first_diff(got, want)))
            continue
        if ctx(mx).decode_stream(want) != O.decode(want):
            bad.append((t, "decode", recs.shape[0], mx))
    assert not bad, bad[:5]


@pytest.mark.parametrize("senders", [255, 257, 700])
def test_many_sources_per_table(senders):
    """Epoch lines with more distinct sources per table than the small LDS hash holds (256)
    take the large-table kernel; the bytes and the footer order stay the reference's."""
    recs = S.gen_stream(senders, 6 * senders, n_sets=1, n_senders=senders, jitter=8)
    want, _ = O.encode(recs, 131072)
    got = ctx(131072).encode_stream(recs)
    assert got == want, first_diff(got, want)
    assert ctx(131072).decode_stream(want) == O.decode(want)


def test_encode_chunk_payload():
    rng = np.random.default_rng(5)
    for t in range(20):
        recs = S.gen_stream(int(rng.integers(1 << 30)), int(rng.integers(1, 2000)), n_sets=int(rng.integers(1, 5)),
                            n_senders=int(rng.integers(2, 30)), jitter=8)
        want, foot = O.encode(recs, 1 << 40)
        payload, ranks = ctx(131072).encode_chunk(recs)
        assert payload == want[8:foot]
        tabs = O.parse_tables(O.decode(want))[0]
        assert list(ranks) == [int(x) for t_ in tabs for x in t_["epoch_rank"]]


@pytest.fixture(scope="module")
def batch():
    p = rempi_amd.default_gen_params(world_size=64, events_per_rank=60000)
    c = ctx(131072)
    d_rec, rec_off = c.generate_device(p, 5, 4)
    host = [rempi_amd.generate_host(p, 5 + r) for r in range(4)]
    return p, c, d_rec, rec_off, host


def test_generator_device_matches_host(batch):
    p, c, d_rec, rec_off, host = batch
    dev = cdcx.d2h(d_rec, int(rec_off[-1]) * 32, np.int32).reshape(-1, 8)
    for r in range(4):
        np.testing.assert_array_equal(dev[rec_off[r]:rec_off[r + 1]], host[r])


def test_batch_encode_decode_vs_oracle(batch):
    p, c, d_rec, rec_off, host = batch
    d_out, off, ln = c.encode_batch_device(d_rec, rec_off)
    files = [cdcx.d2h(d_out + int(off[r]), int(ln[r])).tobytes() for r in range(4)]
    for r in range(4):
        want, _ = O.encode(host[r], 131072)
        assert files[r] == want, (r, first_diff(files[r], want))
    d_keys, n_keys = c.batch_sorted_keys()
    keys = cdcx.d2h(d_keys, n_keys * 8, np.int32).reshape(-1, 2)
    np.testing.assert_array_equal(keys, np.concatenate([O.sorted_keys(h, 131072) for h in host]))
    d_recs, n_recs, d_perm = c.decode_batch_device(d_out, off, ln, d_keys, n_keys)
    tiers = c.decode_tiers()
    assert tiers[1] == 0 and tiers[4] > tiers[0], tiers  # the bench workload stays in the segment tier
    recs = cdcx.d2h(d_recs, n_recs * 32, np.int32).reshape(-1, 8)
    want = np.concatenate([S.expected_table_streams(h, 131072) for h in host])
    np.testing.assert_array_equal(recs, want)


def test_eight_contexts_in_flight_vs_oracle():
    """Eight contexts of one process, one host thread and HIP stream each, encoding and decoding
    different rank traces at the same time (the bench's lanes): the gates, the per-device count of
    calls in flight and the chain kernel's grid that follows it are shared state.  Every file and
    every decoded record stream must be what the same call gives alone."""
    import threading

    p = rempi_amd.default_gen_params(world_size=64, events_per_rank=50000)
    n_lanes, per_lane, rounds = 8, 2, 3
    host = {r: rempi_amd.generate_host(p, r) for r in range(n_lanes * per_lane)}
    want_file = {r: O.encode(h, 131072)[0] for r, h in host.items()}
    want_recs = {r: S.expected_table_streams(h, 131072) for r, h in host.items()}
    errs = []

    def lane(k):
        try:
            c = ctx(131072)
            s = cdcx.stream_create()
            first = k * per_lane
            d_rec, rec_off = c.generate_device(p, first, per_lane, stream=s)
            for _ in range(rounds):
                d_out, off, ln = c.encode_batch_device(d_rec, rec_off, stream=s)
                d_keys, n_keys = c.batch_sorted_keys()
                d_recs, n_recs, _ = c.decode_batch_device(d_out, off, ln, d_keys, n_keys, stream=s)
                cdcx.stream_sync(s)
                for q in range(per_lane):
                    got = cdcx.d2h(d_out + int(off[q]), int(ln[q])).tobytes()
                    if got != want_file[first + q]:
                        errs.append((k, q, "file", first_diff(got, want_file[first + q])))
                recs = cdcx.d2h(d_recs, n_recs * 32, np.int32).reshape(-1, 8)
                if not np.array_equal(recs, np.concatenate([want_recs[first + q] for q in range(per_lane)])):
                    errs.append((k, "records"))
            cdcx.stream_destroy(s)
            c.close()
        except Exception as e:  # noqa: BLE001 - reported on the main thread
            errs.append((k, repr(e)))

    ts = [threading.Thread(target=lane, args=(k,)) for k in range(n_lanes)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs[:4]


def test_verify_roundtrip_with_merged_poll_runs():
    """cdcx_verify_roundtrip_device on traces whose tables merge polls into runs (polls of one
    table that other tables' events separate in the stream): the decoded records are fewer than
    the input records, every run is one record with the summed count, and the check finds a
    single changed word on either side."""
    traces = []
    for seed in (11, 12, 13):
        rng = np.random.default_rng(seed)
        t = S.gen_stream(seed, 2500, n_sets=3, n_senders=6, jitter=8, p_unmatched=0.5, p_group=0.1)
        # extra polls of a table between other tables' records: next to that table's own polls in its stream
        rows = []
        for r in t:
            rows.append(r)
            if r[4] == 0 and rng.random() < 0.3:
                rows.append(np.array([1 + int(rng.integers(7)), 2, 0, 0, 0, 0, 0, (int(r[7]) + 1 + int(rng.integers(2))) % 3], np.int32))
        traces.append(S.canonicalize(np.array(rows, np.int32)))
    rec_off = np.concatenate([[0], np.cumsum([t.shape[0] for t in traces])]).astype(np.int64)
    mx = 700
    dev = cdcx.DeviceArray(np.concatenate(traces))
    c = ctx(mx)
    try:
        d_out, off, ln = c.encode_batch_device(dev.ptr, rec_off)
        d_keys, n_keys = c.batch_sorted_keys()
        d_recs, n_recs, _ = c.decode_batch_device(d_out, off, ln, d_keys, n_keys)
        want = np.concatenate([S.expected_table_streams(t, mx) for t in traces])
        assert n_recs == want.shape[0] < rec_off[-1]  # runs were merged
        np.testing.assert_array_equal(cdcx.d2h(d_recs, n_recs * 32, np.int32).reshape(-1, 8), want)
        assert c.verify_roundtrip_device(dev.ptr) == 0
        # a run's count on the decoded side, then a poll's count on the input side
        k = int(np.flatnonzero((want[:, 2] == 0) & (want[:, 0] > 1))[0])
        word = np.array([want[k, 0] + 1], np.int32)
        assert cdcx.hip().hipMemcpy(d_recs + 32 * k, word.ctypes.data, 4, 1) == 0
        assert c.verify_roundtrip_device(dev.ptr) == 1
        word[0] = want[k, 0]
        assert cdcx.hip().hipMemcpy(d_recs + 32 * k, word.ctypes.data, 4, 1) == 0
        assert c.verify_roundtrip_device(dev.ptr) == 0
        allr = np.concatenate(traces)
        j = int(np.flatnonzero(allr[:, 2] == 0)[5])
        word[0] = allr[j, 0] + 3
        assert cdcx.hip().hipMemcpy(dev.ptr + 32 * j, word.ctypes.data, 4, 1) == 0
        assert c.verify_roundtrip_device(dev.ptr) == 1
    finally:
        dev.close()


@pytest.mark.parametrize("jitter,world,events,max_len", [(0, 64, 40000, 131072), (32, 256, 120000, 131072),
                                                          (128, 1024, 60000, 8192), (8, 4, 30000, 512)])
def test_generator_workloads_vs_oracle(jitter, world, events, max_len):
    """Synthetic traces across jitter (window/segment fallbacks on the device path)."""
    p = rempi_amd.default_gen_params(world_size=world, jitter=jitter, events_per_rank=events)
    c = ctx(max_len)
    d_rec, rec_off = c.generate_device(p, 1, 2)
    d_out, off, ln = c.encode_batch_device(d_rec, rec_off)
    for r in range(2):
        host = rempi_amd.generate_host(p, 1 + r)
        want, _ = O.encode(host, max_len)
        got = cdcx.d2h(d_out + int(off[r]), int(ln[r])).tobytes()
        assert got == want, (r, first_diff(got, want))
        assert c.decode_stream(got) == O.decode(want)


@pytest.mark.parametrize("tier", [0, 1, 2])
def test_chain_tiers_vs_oracle(tier, monkeypatch):
    """Each chain tier alone (16-lane groups, 64-lane groups, lane kernel) reproduces the
    reference bytes; the escalation path is taken when leaf lists outgrow a tier."""
    monkeypatch.setenv("CDCX_CHAIN_TIER", str(tier))
    c = rempi_amd.Context(131072)
    monkeypatch.delenv("CDCX_CHAIN_TIER")
    rng = np.random.default_rng(77 + tier)
    bad = []
    for t in range(60):
        mode = ["jitter", "jitter", "jitter", "reversed", "random"][t % 5]
        recs = S.gen_stream(int(rng.integers(1 << 30)), int(rng.integers(0, 4000)), n_sets=int(rng.integers(1, 4)),
                            n_senders=int(rng.integers(1, 80)), jitter=int(rng.choice([0, 4, 8, 32, 200])), mode=mode)
        want, _ = O.encode(recs, 131072)
        got = c.encode_stream(recs)
        if got != want:
            bad.append((t, mode, recs.shape[0], first_diff(got, want)))
    assert not bad, bad[:5]
    seen = [0, 0, 0]
    for jitter in (8, 32, 128):
        p = rempi_amd.default_gen_params(world_size=256, jitter=jitter, events_per_rank=150000)
        d_rec, rec_off = c.generate_device(p, 3, 2)
        d_out, off, ln = c.encode_batch_device(d_rec, rec_off)
        tiers = c.chain_tiers()
        seen = [a + (b > 0) for a, b in zip(seen, tiers)]
        for r in range(2):
            want, _ = O.encode(rempi_amd.generate_host(p, 3 + r), 131072)
            got = cdcx.d2h(d_out + int(off[r]), int(ln[r])).tobytes()
            assert got == want, (jitter, r, tiers, first_diff(got, want))
    if tier == 0:
        assert seen[1] > 0, "no segment escalated from the 16-lane tier"
    c.close()


def test_chain_g16_first_tier_vs_oracle(monkeypatch):
    """The 16-lane chain kernel as first tier (CDCX_CHAIN_G16: the path a context takes by itself
    when a batch holds 2^30 rows or more, where the 8-lane kernel's 32-bit row offsets end):
    reference bytes on random streams and on the generator workloads, with escalations."""
    monkeypatch.setenv("CDCX_CHAIN_G16", "1")
    c = rempi_amd.Context(131072)
    monkeypatch.delenv("CDCX_CHAIN_G16")
    rng = np.random.default_rng(1234)
    bad = []
    for t in range(40):
        mode = ["jitter", "jitter", "jitter", "reversed", "random"][t % 5]
        recs = S.gen_stream(int(rng.integers(1 << 30)), int(rng.integers(0, 4000)), n_sets=int(rng.integers(1, 4)),
                            n_senders=int(rng.integers(1, 80)), jitter=int(rng.choice([0, 4, 8, 32, 200])), mode=mode)
        want, _ = O.encode(recs, 131072)
        got = c.encode_stream(recs)
        if got != want:
            bad.append((t, mode, recs.shape[0], first_diff(got, want)))
    assert not bad, bad[:5]
    for jitter in (8, 32, 128):
        p = rempi_amd.default_gen_params(world_size=256, jitter=jitter, events_per_rank=150000)
        d_rec, rec_off = c.generate_device(p, 3, 2)
        d_out, off, ln = c.encode_batch_device(d_rec, rec_off)
        kt = c.kernel_times()
        for r in range(2):
            want, _ = O.encode(rempi_amd.generate_host(p, 3 + r), 131072)
            got = cdcx.d2h(d_out + int(off[r]), int(ln[r])).tobytes()
            assert got == want, (jitter, r, c.chain_tiers(), first_diff(got, want))
    c.close()


@pytest.mark.parametrize("tier", [0, 1, 2, 3])
def test_decode_tiers_vs_oracle(tier, monkeypatch):
    """Each permutation-rebuild tier alone (pair segments in 16-lane LDS-ring groups, whole units
    in such groups, 256-slot window, sequential list) reproduces the reference tables and
    records, including streams whose moves reach past the first tiers' window (random /
    reversed permutations) and tables of several pair segments."""
    monkeypatch.setenv("CDCX_DEC_TIER", str(tier))
    c = rempi_amd.Context(131072)
    monkeypatch.delenv("CDCX_DEC_TIER")
    rng = np.random.default_rng(91 + tier)
    bad = []
    for t in range(40):
        mode = ["jitter", "jitter", "jitter", "reversed", "random"][t % 5]
        n = int(rng.integers(0, 3000)) if t % 4 else int(rng.integers(8000, 20000))
        recs = S.gen_stream(int(rng.integers(1 << 30)), n, n_sets=int(rng.integers(1, 4)),
                            n_senders=int(rng.integers(1, 80)), jitter=int(rng.choice([0, 4, 8, 32, 200])), mode=mode)
        want, _ = O.encode(recs, 131072)
        if c.decode_stream(want) != O.decode(want):
            bad.append((t, mode, "tables"))
            continue
        keys = O.sorted_keys(recs, 131072)
        if not np.array_equal(c.reconstruct_stream(want, keys), O.reconstruct(want, keys)):
            bad.append((t, mode, "records"))
    assert not bad, bad[:5]
    c.close()


def test_decode_segment_rerun_vs_oracle():
    """Ranks 317 and 446 of the bench workload at 400 K events each have a pair segment (one in
    about 10^5 has; rank 317 with segments of 1024 pairs, rank 446 with 2048) whose replay of the
    128 pairs before it does not give the state its predecessor ends in: the state check finds
    it, the segment runs again from the predecessor's state, and the tables are the reference's
    without the table leaving the first tier."""
    p = rempi_amd.default_gen_params(world_size=1024, events_per_rank=400_000)
    c = ctx(131072)
    reruns = 0
    for rank in (317, 446):
        recs = rempi_amd.generate_host(p, rank)
        want, _ = O.encode(recs, 131072)
        assert c.decode_stream(want) == O.decode(want)
        tiers = c.decode_tiers()
        assert tiers[1] == 0 and tiers[6] == 0, tiers
        reruns += tiers[5]
        keys = O.sorted_keys(recs, 131072)
        np.testing.assert_array_equal(c.reconstruct_stream(want, keys), O.reconstruct(want, keys))
    assert reruns >= 1


def _moved(n, rng, moves, reach):
    """0..n-1 with `moves` elements taken out and put back up to `reach` places away."""
    order = list(range(n))
    for _ in range(moves):
        i = int(rng.integers(0, n))
        j = int(np.clip(i + rng.integers(-reach, reach + 1), 0, n - 1))
        order.insert(j, order.pop(i))
    return order


@pytest.mark.parametrize("shape", ["dense_near", "dense_far", "sparse_far", "boundary_far", "blocks"])
def test_decode_pair_segments_vs_oracle(shape):
    """Tables whose pair lists span several segments of the permutation rebuild: dense short
    moves (every segment checks out), moves that reach further than a segment replays or than
    its window holds (the unit falls to the whole-unit tiers), a few long moves right where a
    segment starts, and closed blocks of unequal density."""
    rng = np.random.default_rng(len(shape) * 977 + 5)
    c = ctx(131072)
    bad = []
    for t in range(4):
        n = int(rng.integers(6000, 16000))
        if shape == "dense_near":
            order = _moved(n, rng, n, 12)
        elif shape == "dense_far":
            order = _moved(n, rng, n // 2, 150)
        elif shape == "sparse_far":
            order = _moved(n, rng, n // 2, 6)
            for _ in range(8):
                i = int(rng.integers(0, n))
                order.insert(int(np.clip(i + rng.integers(-900, 900), 0, n - 1)), order.pop(i))
        elif shape == "boundary_far":
            order = _moved(n, rng, n, 10)
            want_ids, _ = O.cdc_pairs(np.array(order, np.int32))
            for s in range(1, len(want_ids) // 1024 + 1):  # disturb the list around every 1024th pair's id
                x = int(want_ids[min(s * 1024, len(want_ids) - 1)])
                for dx in (-70, -33, 5, 40):
                    i = order.index(int(np.clip(x + dx, 0, n - 1)))
                    order.insert(int(np.clip(i + rng.integers(-60, 60), 0, n - 1)), order.pop(i))
        else:
            order, base = [], 0
            while base < n:
                L = int(rng.choice([1, 5, 40, 300, 2500]))
                blk = _moved(L, rng, int(L * rng.choice([0.0, 0.3, 1.5])), int(rng.choice([3, 20, 90])))
                order += [base + v for v in blk]
                base += L
        recs = S.permutation_stream(order, src=4)
        want, _ = O.encode(recs, 131072)
        if c.decode_stream(want) != O.decode(want):
            bad.append((shape, t, len(order), "tables"))
            continue
        tiers = c.decode_tiers()
        if shape == "dense_near":
            assert tiers[4] > tiers[0] and tiers[1] == 0, tiers  # several segments, all checked out
        if shape == "dense_far":
            assert tiers[4] > tiers[0] and tiers[1] > 0, tiers  # moves past the window: the table left the first tier
        keys = O.sorted_keys(recs, 131072)
        if not np.array_equal(c.reconstruct_stream(want, keys), O.reconstruct(want, keys)):
            bad.append((shape, t, len(order), "records"))
    assert not bad, bad


@pytest.mark.parametrize("tier", [0, 1])
def test_rank_tiers_vs_oracle(tier, monkeypatch):
    """Clock-order rank: the windowed pass (tier 0; units it cannot rank take the tile sort)
    and the tile sort alone (tier 1) give the reference bytes, on multi-tile tables of every
    arrival mode and on sorted streams with one event moved by about D and 2D (window D = 64),
    on either side of a tile boundary."""
    monkeypatch.setenv("CDCX_RANK_TIER", str(tier))
    c = rempi_amd.Context(131072)
    monkeypatch.delenv("CDCX_RANK_TIER")
    rng = np.random.default_rng(505 + tier)
    bad = []
    for t in range(30):
        mode = ["jitter", "jitter", "sorted", "reversed", "random"][t % 5]
        recs = S.gen_stream(int(rng.integers(1 << 30)), int(rng.integers(1, 6000)), n_sets=int(rng.integers(1, 3)),
                            n_senders=int(rng.integers(1, 60)), jitter=int(rng.choice([0, 8, 24, 64, 400])), mode=mode)
        want, _ = O.encode(recs, 131072)
        got = c.encode_stream(recs)
        if got != want:
            bad.append((t, mode, first_diff(got, want)))
    base = S.gen_stream(99, 3000, n_sets=1, n_senders=16, mode="sorted", p_unmatched=0.0, p_group=0.0)
    for k in (31, 63, 64, 65, 66, 127, 128, 129, 130, -65, -129):
        for i in (500, 1000, 1030, 2040):
            r = list(base)
            e = r.pop(i)
            r.insert(min(max(i + k, 0), len(r)), e)
            recs = S.canonicalize(np.array(r))
            want, _ = O.encode(recs, 131072)
            got = c.encode_stream(recs)
            if got != want:
                bad.append(("move", i, k, first_diff(got, want)))
    assert not bad, bad[:5]
    c.close()


@pytest.mark.parametrize("reach", [12, 45, 300, 1500])
def test_chain_deep_levels_vs_oracle(reach):
    """Long rising runs with elements displaced up to `reach` places: new nodes land far below
    the top level, so the chain kernel searches and updates the spilled tops -- the eight levels
    in registers, the LDS ring of the last 32 spilled levels and the lines already written to
    memory -- and the edit sequence has entries far from their column's stretch."""
    rng = np.random.default_rng(1000 + reach)
    c = ctx(131072)
    bad = []
    for t in range(6):
        n = int(rng.integers(1500, 6000))
        order = list(range(n))
        for _ in range(n // 25):  # move 4 % of the elements up to `reach` places
            i = int(rng.integers(0, n))
            j = int(np.clip(i + rng.integers(-reach, reach + 1), 0, n - 1))
            order.insert(j, order.pop(i))
        recs = S.permutation_stream(order, src=3)
        want, _ = O.encode(recs, 131072)
        got = c.encode_stream(recs)
        if got != want:
            bad.append((t, n, first_diff(got, want)))
        elif c.decode_stream(got) != O.decode(want):
            bad.append((t, n, "tables"))
    assert not bad, bad


def _stitch_blocks(kind, rng):
    """Blocks that are closed prefixes (segments) of one table's permutation, of a given shape."""
    pool = [1, 2, 63, 64, 65, 130, 255, 256, 257, 700, 1500]
    if kind in ("saw", "rise_then_fall"):  # (thousands of open lists at once run in the slowest chain tier)
        pool.append(6000)
    sizes = [int(x) for x in rng.choice(pool, size=int(rng.integers(4, 9)))]
    out, base = [], 0
    for L in sizes:
        if kind == "falling":  # every row ends a list of its own
            blk = list(range(L - 1, -1, -1))
        elif kind == "rise_then_fall":  # a rising run, then many rows that all end at the top level
            k = max(1, L // 3)
            blk = list(range(k)) + list(range(L - 1, k - 1, -1))
        elif kind == "fall_then_rise":
            k = max(1, L // 2)
            blk = list(range(L - 1, L - 1 - k, -1)) + list(range(L - k))
        elif kind == "saw":  # short falling teeth on a rising line, under one long edge
            blk = []
            t = int(rng.integers(2, 9))
            for a in range(0, L - 1, t):
                blk += list(range(min(a + t, L - 1) - 1, a - 1, -1))
            blk = [L - 1] + blk
        else:  # random
            blk = [int(x) for x in rng.permutation(L)]
        assert sorted(blk) == list(range(L)), (kind, L)
        out += [base + v for v in blk]
        base += L
    return out


@pytest.mark.parametrize("kind", ["falling", "rise_then_fall", "fall_then_rise", "saw", "random"])
def test_chain_stitching_shapes_vs_oracle(kind):
    """Segments with many max-level rows (more than a wave has lanes), with many rows whose
    outside parent comes from an anchor, and of lengths on either side of the 64-row chunks
    and 256-row groups in which the exits are swept; the permutation and its inverse."""
    rng = np.random.default_rng(len(kind) * 131 + 7)
    c = ctx(131072)
    bad = []
    for t in range(5):
        order = _stitch_blocks(kind, rng)
        inv = [0] * len(order)
        for i, v in enumerate(order):
            inv[v] = i
        for which, perm in (("perm", order), ("inverse", inv)):
            recs = S.permutation_stream(perm, src=2)
            want, _ = O.encode(recs, 131072)
            got = c.encode_stream(recs)
            if got != want:
                bad.append((t, which, len(perm), first_diff(got, want)))
            elif c.decode_stream(got) != O.decode(want):
                bad.append((t, which, len(perm), "tables"))
    assert not bad, bad


@pytest.mark.parametrize("n_sets", [17, 64, 200, 256])
def test_many_tables_vs_oracle(n_sets):
    """Ranks with many matching sets: table indexes of up to eight bits in the scatter's ballots,
    the high rows of its slot table and of the tile histograms, hundreds of units per chunk."""
    rng = np.random.default_rng(4000 + n_sets)
    bad = []
    for t, mx in enumerate((131072, 131072, 700)):
        ids = sorted(int(x) for x in rng.choice(256, size=n_sets, replace=False))
        recs = S.gen_stream(int(rng.integers(1 << 30)), int(rng.integers(2000, 6000)), n_senders=n_sets + int(rng.integers(0, 20)),
                            set_ids=ids, jitter=6)
        want, _ = O.encode(recs, mx)
        got = ctx(mx).encode_stream(recs)
        if got != want:
            bad.append((t, mx, recs.shape[0], first_diff(got, want)))
        elif ctx(mx).decode_stream(got) != O.decode(want):
            bad.append((t, mx, "tables"))
    assert not bad, bad


def test_set_id_out_of_range():
    """matching_set_id 256 is past the library's limit: an error, not a wrong file."""
    recs = S.gen_stream(11, 500, n_senders=6, set_ids=[0, 3, 256])
    with pytest.raises(cdcx.CdcxError):
        ctx(131072).encode_stream(recs)
