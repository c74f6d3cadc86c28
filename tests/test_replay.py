"""Replay-side streaming decode: cdcx_replay_decode_files over a
REMPI_DIR of rank files must hand every file's tables to the sink exactly as
cdcx_decode_stream / the reference decode() produce them for that file alone, whatever
the batching and the number of contexts.  Rank files are the reference-written golden
fixtures plus oracle-encoded synthetic streams."""
import os

import numpy as np
import pytest

import cdc_streams as S
import golden_util as G
import oracle_lib as O
from rempi_amd import cdcx, replay

OK_NAMES = [n for n in G.names() if not G.load(n)["ref_failed"]]


def test_rank_files_order_and_filter(tmp_path):
    for name in ["rank_10.rempi", "rank_2.rempi", "rank_0.rempi", "rank_x.rempi", "rank_3.rempi.gz", "notes.txt"]:
        (tmp_path / name).write_bytes(b"")
    got = replay.rank_files(str(tmp_path))
    assert [r for r, _ in got] == [0, 2, 10]
    assert all(os.path.basename(p) == f"rank_{r}.rempi" for r, p in got)
    assert [r for r, _ in replay.rank_files(str(tmp_path), range(1, 10))] == [2]


def test_replay_entry_point_declared():
    assert "cdcx_replay_decode_files" in cdcx.exported_symbols()


def _rempi_dir(tmp_path, n_synth=6):
    """rank_<r>.rempi files: the golden fixtures, then synthetic streams; -> {rank: tables}."""
    want = {}
    r = 0
    for name in OK_NAMES:
        d = G.load(name)
        (tmp_path / f"rank_{r}.rempi").write_bytes(d["rempi"])
        want[r] = d["tables"]
        r += 1
    for k in range(n_synth):
        recs = S.gen_stream(seed=900 + k, n_matched=3000 + 1700 * k, n_sets=1 + k % 3, jitter=2 + 3 * k)
        data, _ = O.encode(recs, 1024 if k % 2 else 131072)
        (tmp_path / f"rank_{r}.rempi").write_bytes(data)
        want[r] = O.decode(data)
        r += 1
    return want


@pytest.mark.gpu
@pytest.mark.parametrize("streams,batch_bytes", [(1, 0), (2, 1), (3, 4096), (4, 1 << 16)])
def test_replay_dir_matches_per_file_decode(tmp_path, streams, batch_bytes):
    want = _rempi_dir(tmp_path)
    got = {}

    def sink(rank, data):
        assert rank not in got
        got[rank] = data

    st, ranks = replay.decode_dir(str(tmp_path), streams=streams, batch_bytes=batch_bytes, sink=sink)
    assert sorted(got) == sorted(want) == ranks
    for r in want:
        assert got[r] == want[r], r
    assert st["files"] == len(want)
    assert st["file_bytes"] == sum(os.path.getsize(tmp_path / f"rank_{r}.rempi") for r in want)
    if batch_bytes == 1:
        assert st["batches"] == len(want)


@pytest.mark.gpu
def test_replay_gzip_dir(tmp_path):
    want = {}
    for r, name in enumerate(G.gzip_names()):
        d = G.load_gzip(name)
        (tmp_path / f"rank_{r}.rempi").write_bytes(d["rempi_gz"])
        want[r] = d["tables"]
    got = {}
    replay.decode_dir(str(tmp_path), streams=2, batch_bytes=1, gzip=1, sink=lambda r, b: got.__setitem__(r, b))
    assert got == want


@pytest.mark.gpu
def test_replay_corrupt_file_fails_loudly(tmp_path):
    want = _rempi_dir(tmp_path, n_synth=2)
    bad = bytearray((tmp_path / "rank_1.rempi").read_bytes())
    bad[:8] = np.uint64(1 << 40).tobytes()  # first chunk length past the end of the file
    (tmp_path / "rank_1.rempi").write_bytes(bytes(bad))
    assert len(want) > 2
    with pytest.raises(cdcx.CdcxError) as e:
        replay.decode_dir(str(tmp_path), streams=2, batch_bytes=1)
    assert e.value.code == 4


@pytest.mark.gpu
def test_replay_sink_error_stops_pipeline(tmp_path):
    _rempi_dir(tmp_path, n_synth=2)

    def sink(rank, data):
        raise ValueError("consumer failed")

    with pytest.raises(ValueError):
        replay.decode_dir(str(tmp_path), streams=2, batch_bytes=1, sink=sink)


@pytest.mark.gpu
def test_replay_cli_writes_tables(tmp_path):
    want = _rempi_dir(tmp_path / "in" if (tmp_path / "in").mkdir() is None else None, n_synth=1)
    assert replay.main([str(tmp_path / "in"), "--streams", "2", "--out", str(tmp_path / "out")]) == 0
    for r, t in want.items():
        assert (tmp_path / "out" / f"rank_{r}.tables").read_bytes() == t


def _as_chunks(dump: bytes):
    """Reference table dump -> per chunk, per table the fields as comparable python values."""
    out = []
    for ch in O.parse_tables(dump):
        out.append([{k: (t[k].tolist() if hasattr(t[k], "tolist") else t[k]) for k in t} for t in ch])
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("streams,batch_bytes", [(1, 0), (3, 4096)])
def test_replay_dir_delivers_reference_tables(tmp_path, streams, batch_bytes):
    """cdcx_replay_decode_tables: the flat tables handed to the sink (pointers into the pinned
    buffers, no host formatting) hold exactly what the reference decode() leaves in each chunk's
    test tables."""
    want = _rempi_dir(tmp_path, n_synth=3)
    got = {}

    def sink(rank, chunks):
        got[rank] = chunks

    st, ranks = replay.decode_dir_tables(str(tmp_path), streams=streams, batch_bytes=batch_bytes, sink=sink)
    assert sorted(got) == sorted(want) == ranks
    for r in want:
        ref = _as_chunks(want[r])
        assert len(got[r]) == len(ref), r
        for gch, rch in zip(got[r], ref):
            assert [t["set_id"] for t in gch] == [t["set_id"] for t in rch]
            for g, w in zip(gch, rch):
                assert g["count"] == w["count"]
                for k in ("epoch_rank", "epoch_clock", "with_previous", "matched_index", "ids", "delays", "perm"):
                    assert g[k].tolist() == w[k], (r, k)
                um = dict(zip(g["unmatched_id"].tolist(), g["unmatched_count"].tolist()))
                assert sorted(um.items()) == [tuple(x) for x in w["unmatched"]], r
    assert st["files"] == len(want)


@pytest.mark.gpu
def test_replay_rejects_a_context_passed_twice(tmp_path):
    _rempi_dir(tmp_path, n_synth=1)
    c = cdcx.Context()
    with pytest.raises(cdcx.CdcxError) as e:
        cdcx.replay_decode_files([c, c], [p for _, p in replay.rank_files(str(tmp_path))])
    assert e.value.code == 1
    c.close()


@pytest.mark.gpu
def test_replay_1024_files_over_4_contexts(tmp_path):
    """1024 small rank files of the bench workload through four contexts in small batches: every
    file's tables arrive once, and their permutated indices are the ones cdcx_decode_batch_device
    gives for the same file right after encoding; two of the files also against the oracle."""
    import hashlib

    import rempi_amd

    n_files, per = 1024, 128
    p = cdcx.default_gen_params(world_size=1024, events_per_rank=3000)
    ctx = cdcx.Context()
    want, keep = {}, {}
    for b0 in range(0, n_files, per):
        d_rec, rec_off = ctx.generate_device(p, b0, per)
        d_out, off, ln = ctx.encode_batch_device(d_rec, rec_off)
        img = cdcx.d2h(d_out, int(off[-1] + ln[-1]))
        _, _, d_perm = ctx.decode_batch_device(d_out, off, ln)
        _, po = ctx.decode_rank_offsets(per)
        perm = cdcx.d2h(d_perm, int(po[-1]) * 4, np.int32)
        for i in range(per):
            data = img[off[i]:off[i] + ln[i]].tobytes()
            (tmp_path / f"rank_{b0 + i}.rempi").write_bytes(data)
            want[b0 + i] = hashlib.sha256(memoryview(np.ascontiguousarray(perm[po[i]:po[i + 1]]))).hexdigest()
            if b0 + i in (5, 777):
                keep[b0 + i] = data
    ctx.close()
    got = {}

    def sink(rank, chunks):
        assert rank not in got
        h = hashlib.sha256()
        for tabs in chunks:
            for t in tabs:
                h.update(memoryview(np.ascontiguousarray(t["perm"], dtype=np.int32)))
        got[rank] = h.hexdigest()

    st, ranks = replay.decode_dir_tables(str(tmp_path), streams=4, batch_bytes=3 << 20, sink=sink)
    assert st["files"] == n_files and st["batches"] >= 8 and ranks == list(range(n_files))
    assert got == want
    for r, data in keep.items():
        assert data == O.encode(rempi_amd.generate_host(p, r), 131072)[0]
        h = hashlib.sha256()
        for chunk in O.parse_tables(O.decode(data)):
            for t in chunk:
                h.update(memoryview(np.ascontiguousarray(t["perm"], dtype=np.int32)))
        assert h.hexdigest() == want[r]
