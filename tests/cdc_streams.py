"""Random canonical record streams for parity tests (test infrastructure only).

A record is the reference's 8 x int32 test event (rempi_event.h:40-48):
  [0] event_count [1] type (2 = TEST) [2] flag [3] rank/source [4] with_next
  [5] index [6] msg_id = Lamport clock [7] matching_set_id

Streams produced here are *canonical*: they are what rempi_event_list::push
(rempi_event_list.cpp:66-99) hands to the encoder, i.e. no two consecutive records are
equal in fields 1..7 (the run-length merge has already been applied).  `canonicalize`
applies that merge to an arbitrary stream.
"""
from __future__ import annotations

import numpy as np

TEST = 2


def canonicalize(recs: np.ndarray) -> np.ndarray:
    """rempi_event_list::push merge: a record equal to its predecessor in fields 1..7
    bumps the predecessor's event_count by one and is dropped (rempi_event_list.cpp:85-89)."""
    recs = np.asarray(recs, dtype=np.int32).reshape(-1, 8)
    out = []
    for r in recs:
        if out and np.array_equal(out[-1][1:8], r[1:8]):
            out[-1][0] += 1
        else:
            out.append(r.copy())
    return np.array(out, dtype=np.int32).reshape(-1, 8)


def gen_stream(seed: int, n_matched: int, n_sets: int = 2, n_senders: int = 8, jitter: int = 4,
               p_unmatched: float = 0.2, p_group: float = 0.1, mode: str = "jitter",
               max_count: int = 63, index_mod: int = 16, rank_base: int = 0,
               set_ids=None, neg_index: bool = False) -> np.ndarray:
    """Near-sorted (or adversarial, per `mode`) canonical stream of one rank.

    mode: 'jitter' arrival = clock + U[0, jitter]; 'sorted'; 'reversed' (arrival order is
    reverse clock order); 'random' (uniformly random arrival order).
    """
    rng = np.random.default_rng(seed)
    if set_ids is None:
        set_ids = list(range(n_sets))
    n_senders = max(n_senders, 1)
    senders = [rank_base + 1 + j for j in range(n_senders)]
    sender_set = [set_ids[j % len(set_ids)] for j in range(n_senders)]
    clk = np.full(n_senders, 10, dtype=np.int64)
    msgs = []  # (arrival_key, tiebreak, src, clock, set)
    for m in range(n_matched):
        j = int(rng.integers(n_senders))
        clk[j] += 1 + int(rng.integers(8))
        c = int(clk[j])
        if mode == "jitter":
            key = c + int(rng.integers(jitter + 1))
        elif mode == "sorted":
            key = c
        elif mode == "reversed":
            key = -c
        elif mode == "random":
            key = int(rng.integers(1 << 30))
        else:
            raise ValueError(mode)
        msgs.append((key, m, senders[j], c, sender_set[j]))
    msgs.sort()
    queues = {s: [] for s in set_ids}
    for k, (_, _, src, c, s) in enumerate(msgs):
        queues[s].append((k, src, c))
    heads = {s: 0 for s in set_ids}
    taken = np.zeros(len(msgs), dtype=bool)
    recs = []
    k = 0
    while k < len(msgs):
        if taken[k]:
            k += 1
            continue
        s = msgs[k][4]
        if rng.random() < p_unmatched:
            cnt = 1 + min(int(rng.geometric(0.5)) - 1, max_count - 1)
            recs.append([cnt, TEST, 0, 0, 0, 0, 0, s])
        g = 1
        if rng.random() < p_group:
            g = int(rng.integers(2, 5))
        q = queues[s]
        members = []
        while len(members) < g and heads[s] < len(q):
            kk, src, c = q[heads[s]]
            heads[s] += 1
            if taken[kk]:
                continue
            taken[kk] = True
            members.append((src, c))
        for i, (src, c) in enumerate(members):
            idx = int(rng.integers(index_mod))
            if neg_index and rng.random() < 0.05:
                idx = -1 - idx
            recs.append([1, TEST, 1, src, 1 if i + 1 < len(members) else 0, idx, c, s])
        k += 1
    if rng.random() < p_unmatched:  # trailing poll
        recs.append([1 + int(rng.integers(5)), TEST, 0, 0, 0, 0, 0, set_ids[0]])
    return canonicalize(np.array(recs, dtype=np.int32).reshape(-1, 8))


def kat_stream() -> np.ndarray:
    """Known-answer input of test/rempi/rempi_test_compress.cpp:104-113 (rank 1, clocks
    32,11,17,36,31,12,22,10,16,18) framed as a recorder would: 5 polls, the 10 matched
    receives, 3 polls (already run-length merged)."""
    recs = [[5, TEST, 0, 0, 0, 0, 0, 0]]
    for c in [32, 11, 17, 36, 31, 12, 22, 10, 16, 18]:
        recs.append([1, TEST, 1, 1, 0, 0, c, 0])
    recs.append([3, TEST, 0, 0, 0, 0, 0, 0])
    return np.array(recs, dtype=np.int32)


def permutation_stream(c, src: int = 1, set_id: int = 0) -> np.ndarray:
    """A single-table stream whose clock-order permutation is exactly `c`
    (observed row i carries clock 10 + c[i] from one source)."""
    recs = [[1, TEST, 1, src, 0, 0, 10 + int(v), set_id] for v in c]
    return np.array(recs, dtype=np.int32).reshape(-1, 8)


def chunk_bounds(recs: np.ndarray, max_len: int):
    """[(start, end_exclusive)] of the chunks extract_encoder_input_format_chunk cuts
    (rempi_encoder_cdc.cpp:740-778, length rule of add() :178-218)."""
    recs = np.asarray(recs, dtype=np.int32).reshape(-1, 8)
    out = []
    pos, n = 0, recs.shape[0]
    while pos < n:
        start, length, last = pos, 0, None
        last_kind = {}  # set id -> 'm' or 'u' (last record of that table in this chunk)
        while pos < n:
            if last is not None and length > max_len and last[4] == 0:
                break
            r = recs[pos]
            s = int(r[7])
            if r[2] == 1:
                length += 1
                last_kind[s] = "m"
            else:
                if last_kind.get(s) != "u":
                    length += 1
                last_kind[s] = "u"
            last = r
            pos += 1
        out.append((start, pos))
    return out


def expected_table_streams(recs: np.ndarray, max_len: int) -> np.ndarray:
    """Decoded-record parity target: per chunk, per table in
    ascending set id, the table's records in observed order as the decoder can rebuild them
    -- consecutive unmatched polls of a table merged (counts summed, add() :205-208),
    unmatched fields other than count/type/set zeroed, with_next normalised to 0/1, matched
    event_count 1."""
    recs = np.asarray(recs, dtype=np.int32).reshape(-1, 8)
    out = []
    for a, b in chunk_bounds(recs, max_len):
        ch = recs[a:b]
        for s in sorted(set(int(x) for x in ch[:, 7])):
            prev_unmatched = False
            for r in ch[ch[:, 7] == s]:
                if r[2] == 1:
                    out.append([1, 2, 1, r[3], 1 if r[4] != 0 else 0, r[5], r[6], s])
                    prev_unmatched = False
                else:
                    if prev_unmatched:
                        out[-1][0] = np.int32(np.int64(out[-1][0]) + np.int64(r[0]))
                    else:
                        out.append([r[0], 2, 0, 0, 0, 0, 0, s])
                    prev_unmatched = True
    return np.array(out, dtype=np.int32).reshape(-1, 8)


def chunk_bounds_fast(recs: np.ndarray, max_len: int):
    """chunk_bounds with array operations per chunk (full-size traces): the length rule of
    add() (rempi_encoder_cdc.cpp:178-218) as a cumulative sum over a window that is sure to
    hold the chunk's end."""
    recs = np.asarray(recs, dtype=np.int32).reshape(-1, 8)
    n = recs.shape[0]
    matched = recs[:, 2] == 1
    out, start = [], 0
    while start < n:
        win = max(2 * max_len + 64, 1024)
        while True:
            end = min(n, start + win)
            m = matched[start:end]
            s = recs[start:end, 7]
            order = np.argsort(s, kind="stable")
            so = s[order]
            prev = np.full(end - start, -1, dtype=np.int64)  # previous record of the same set in the window
            same = np.zeros(end - start, dtype=bool)
            same[1:] = so[1:] == so[:-1]
            prev[order[1:]] = np.where(same[1:], order[:-1], -1)
            prev_unmatched = np.zeros(end - start, dtype=bool)
            has = prev >= 0
            prev_unmatched[has] = ~m[prev[has]]
            inc = np.where(m, 1, np.where(prev_unmatched, 0, 1))
            length = np.cumsum(inc)
            close = np.nonzero((length > max_len) & (recs[start:end, 4] == 0))[0]
            if close.size:
                stop = start + int(close[0]) + 1
                break
            if end == n:
                stop = n
                break
            win *= 2
        out.append((start, stop))
        start = stop
    return out


def expected_table_streams_fast(recs: np.ndarray, max_len: int) -> np.ndarray:
    """expected_table_streams with array operations (full-size traces)."""
    recs = np.asarray(recs, dtype=np.int32).reshape(-1, 8)
    parts = []
    for a, b in chunk_bounds_fast(recs, max_len):
        ch = recs[a:b]
        ch = ch[np.argsort(ch[:, 7], kind="stable")]  # per table, observed order
        m = ch[:, 2] == 1
        # an unmatched record continues a run when the record before it (same table) is unmatched
        cont = np.zeros(ch.shape[0], dtype=bool)
        cont[1:] = (~m[1:]) & (~m[:-1]) & (ch[1:, 7] == ch[:-1, 7])
        head = ~cont
        gid = np.cumsum(head) - 1
        out = np.zeros((int(head.sum()), 8), dtype=np.int32)
        hm = m[head]
        hrec = ch[head]
        out[:, 1] = 2
        out[:, 7] = hrec[:, 7]
        out[hm, 0] = 1
        out[hm, 2] = 1
        out[hm, 3] = hrec[hm, 3]
        out[hm, 4] = (hrec[hm, 4] != 0).astype(np.int32)
        out[hm, 5] = hrec[hm, 5]
        out[hm, 6] = hrec[hm, 6]
        cnt = np.zeros(out.shape[0], dtype=np.int64)
        np.add.at(cnt, gid[~m], ch[~m, 0].astype(np.int64))
        out[~hm, 0] = cnt[~hm].astype(np.int32)  # wraps like the reference's int add
        parts.append(out)
    return np.concatenate(parts) if parts else np.zeros((0, 8), np.int32)
