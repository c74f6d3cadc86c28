"""Damaged rank files on the replay side: every section-size word of the reference-written
golden files (epoch, with_previous, matched_index, unmatched ids, unmatched counts, pairs;
decode, rempi_encoder_cdc.cpp:1044-1200) is overwritten in turn.  The reference reports
damage with "Record data is broken" (:952, :1288) or reads out of bounds; the device
decoder must either return CDCX_ERR_CORRUPT or produce exactly the tables the CPU oracle
produces from the same damaged bytes -- and never write outside a unit's scratch rows."""
import numpy as np
import pytest

import golden_util as G
import oracle_lib as O
import rempi_amd
from rempi_amd import cdcx

FILES = ["kat", "multichunk_small_max", "unmatched_heavy", "groups_heavy", "s200_jitter4_t2_m16", "s1000_jitter0_t4_m131072",
         "sparse_set_ids"]


def size_word_offsets(data: bytes, limit_units=6):
    """Byte offsets of the six section-size words of the first units of every chunk."""
    out = []
    u64 = lambda p: int(np.frombuffer(data[p:p + 8], np.uint64)[0])  # noqa: E731
    p = 0
    while True:
        n = u64(p)
        p += 8
        if n == 0:
            break
        q, end, k = p, p + n, 0
        while q < end and k < limit_units:
            words = {}
            words["esz"] = q + 8
            q2 = q + 16 + 2 * u64(q + 8)
            words["wsz"] = q2 + 8
            q2 += 16 + u64(q2 + 8)
            words["msz"] = q2 + 8
            q2 += 16 + u64(q2 + 8)
            words["usz"] = q2
            q2 += 8 + u64(q2)
            words["csz"] = q2
            q2 += 8 + u64(q2)
            words["psz"] = q2
            q2 += 8 + u64(q2)
            out.append(words)
            q = q2
            k += 1
        p = end
    return out


def mutations(old):
    return sorted({0, max(old - 8, 0), old + 8, old + 16, 2 * old + 8, old + 4, 1 << 40, (1 << 64) - 8} - {old})


@pytest.mark.gpu
@pytest.mark.parametrize("name", FILES)
def test_section_size_mutations(name):
    d = G.load(name)
    data = d["rempi"]
    c = rempi_amd.Context(d["max_len"])
    assert c.decode_stream(data) == d["tables"]
    n_corrupt = n_equal = 0
    for words in size_word_offsets(data)[:4]:
        for field, off in words.items():
            old = int(np.frombuffer(data[off:off + 8], np.uint64)[0])
            for new in mutations(old):
                bad = data[:off] + np.uint64(new).tobytes() + data[off + 8:]
                try:
                    got = c.decode_stream(bad)
                except cdcx.CdcxError as e:
                    assert e.code == 4, (name, field, old, new, e)
                    n_corrupt += 1
                    continue
                try:
                    want = O.decode(bad)
                except O.OracleError:
                    pytest.fail(f"{name} {field} {old}->{new}: oracle rejects, device accepted")
                assert got == want, (name, field, old, new)
                n_equal += 1
    assert n_corrupt > 0
    # the context still decodes the undamaged file afterwards
    assert c.decode_stream(data) == d["tables"]
    c.close()
