"""The entry point that allocates nothing (cdcx_decode_chunk_perm_static: one chunk payload in
device memory -> the tables' permutated indices, all scratch in the library's static device
array) against the existing cdcx_decode_batch_device on the same chunk and against the CPU
oracle's permutated indices, bit for bit: calls in a row on one context, each smaller or
different from the last, so stale scratch would show."""
import numpy as np
import pytest

import cdc_streams as S
import oracle_lib as O
import rempi_amd
from rempi_amd import cdcx

pytestmark = pytest.mark.gpu


def payload_of(recs, max_len=1 << 40):
    """One-chunk CDC payload of a stream (CPU oracle bytes)."""
    data, foot = O.encode(recs, max_len)
    n = int(np.frombuffer(data[:8], np.uint64)[0])
    assert 8 + n == foot, "stream does not fit one chunk"
    return data[8:8 + n], data


def perm_existing(c, data):
    """cdcx_decode_batch_device (tables only) on the one-chunk rank file."""
    buf = np.frombuffer(data, np.uint8)
    pad = np.zeros((-buf.size) % 8, np.uint8)
    d = cdcx.DeviceArray(np.concatenate([buf, pad]))
    _, _, d_perm = c.decode_batch_device(d.ptr, np.array([0], np.int64), np.array([buf.size], np.int64))
    _, po = c.decode_rank_offsets(1)
    out = cdcx.d2h(d_perm, int(po[1]) * 4, np.int32).copy()
    d.close()
    return out


def perm_oracle(data):
    """The oracle's matched_events_permutated_indices of the file's tables, in file order."""
    tabs = [t for chunk in O.parse_tables(O.decode(data)) for t in chunk]
    return np.concatenate([t["perm"] for t in tabs] + [np.zeros(0, np.int64)]).astype(np.int32)


def perm_static(c, payload, d_perm, cap):
    d = cdcx.DeviceArray(np.frombuffer(payload, np.uint8))
    n = c.decode_chunk_perm_static(d.ptr, len(payload), d_perm.ptr, cap)
    out = cdcx.d2h(d_perm.ptr, n * 4, np.int32).copy()
    d.close()
    return out


def test_static_entry_point_matches_batch_decode():
    c = rempi_amd.Context(1 << 40)
    cap = 262144
    d_perm = cdcx.DeviceArray(np.full(cap, -7, np.int32))
    p = rempi_amd.default_gen_params(world_size=64, events_per_rank=120000)
    streams = [
        rempi_amd.generate_host(p, 9),                                             # one large chunk, 4 tables
        S.gen_stream(5, 3000, n_sets=3, n_senders=12, jitter=8),                   # then a much smaller one
        S.gen_stream(6, 2500, n_sets=2, n_senders=9, mode="random"),               # window / list tiers
        S.gen_stream(7, 1800, n_sets=1, n_senders=5, mode="reversed"),
        S.gen_stream(8, 40, n_sets=4, n_senders=3, jitter=2, p_unmatched=0.9),
        np.array([[3, 2, 0, 0, 0, 0, 0, 5]], np.int32),                            # no matched event at all
        rempi_amd.generate_host(p, 10),
    ]
    for k, recs in enumerate(streams):
        payload, data = payload_of(recs)
        want = perm_existing(c, data)
        got = perm_static(c, payload, d_perm, cap)
        assert got.shape == want.shape, (k, got.shape, want.shape)
        np.testing.assert_array_equal(got, want, err_msg=f"stream {k}")
        np.testing.assert_array_equal(got, perm_oracle(data), err_msg=f"stream {k} against the oracle")
    # limits and damage are reported, and the next call still works
    big = rempi_amd.generate_host(rempi_amd.default_gen_params(world_size=64, events_per_rank=330000), 2)
    payload, _ = payload_of(big)
    with pytest.raises(cdcx.CdcxError) as e:
        perm_static(c, payload, d_perm, cap)
    assert e.value.code == 6
    small, data = payload_of(streams[1])
    with pytest.raises(cdcx.CdcxError) as e:
        perm_static(c, small, d_perm, 10)  # caller's buffer too small
    assert e.value.code == 6
    with pytest.raises(cdcx.CdcxError) as e:
        perm_static(c, small[:-8], d_perm, cap)
    assert e.value.code == 4
    np.testing.assert_array_equal(perm_static(c, small, d_perm, cap), perm_existing(c, data))
    # arguments the kernels cannot read are refused: a payload that is not 8-byte aligned, a gzip context
    d = cdcx.DeviceArray(np.frombuffer(b"\0\0\0\0" + small, np.uint8))
    with pytest.raises(cdcx.CdcxError) as e:
        c.decode_chunk_perm_static(d.ptr + 4, len(small), d_perm.ptr, cap)
    assert e.value.code == 1
    d.close()
    cz = rempi_amd.Context(1 << 40, gzip=1)
    with pytest.raises(cdcx.CdcxError) as e:
        perm_static(cz, small, d_perm, cap)
    assert e.value.code == 1
    cz.close()
    # a second context on the same device shares the device's array
    c2 = rempi_amd.Context(1 << 40)
    np.testing.assert_array_equal(perm_static(c2, small, d_perm, cap), perm_existing(c, data))
    c2.close()
    d_perm.close()
    c.close()
