"""The permutation rebuild's pair-segment tier, as a host model (tests/seg_model.py) against the
oracle's cdc_prepare_decode_indices: whenever every segment of a unit finishes and passes the
state check, the permutation is the sequential replay's; when not, the model says so (the
device sends such units to the whole-unit tiers).  CPU only."""
import numpy as np
import pytest

import oracle_lib as O
import seg_model as SM


def moved(n, rng, moves, reach):
    order = list(range(n))
    for _ in range(moves):
        i = int(rng.integers(0, n))
        j = int(np.clip(i + rng.integers(-reach, reach + 1), 0, n - 1))
        order.insert(j, order.pop(i))
    return order


def check(order):
    c = np.array(order, np.int32)
    ids, dl = O.cdc_pairs(c)
    want = O.decode_perm(ids, dl, len(order))
    got = SM.rebuild(ids, dl, len(order))
    if got is not None:
        assert got == [int(v) for v in want]
    return got is not None, SM.nseg(len(ids))


@pytest.mark.parametrize("reach,expect_pass", [(6, True), (12, True), (40, None), (150, None), (2000, None)])
def test_segments_vs_sequential_replay(reach, expect_pass):
    rng = np.random.default_rng(17 + reach)
    passed = multi = 0
    for t in range(6):
        n = int(rng.integers(5000, 12000))
        ok, ns = check(moved(n, rng, n, reach))
        passed += ok
        multi += ns > 1
    assert multi == 6  # (several segments each: the check between them ran)
    if expect_pass:
        assert passed == 6


def test_far_moves_at_segment_starts():
    """Long moves placed where segments start: the replay before a segment cannot rebuild the
    state there, the check has to notice."""
    rng = np.random.default_rng(4)
    outcomes = set()
    for t in range(8):
        n = int(rng.integers(6000, 10000))
        order = moved(n, rng, n, 10)
        ids, _ = O.cdc_pairs(np.array(order, np.int32))
        for s in range(1, len(ids) // SM.PAIRS + 1):
            x = int(ids[min(s * SM.PAIRS, len(ids) - 1)])
            for dx in (-70, -33, 5, 40):
                i = order.index(int(np.clip(x + dx, 0, n - 1)))
                order.insert(int(np.clip(i + rng.integers(-200, 200), 0, n - 1)), order.pop(i))
        outcomes.add(check(order)[0])
    assert False in outcomes  # (some of these must have been refused, else the test is too tame)


def test_small_and_degenerate():
    rng = np.random.default_rng(9)
    for order in ([], [0], [1, 0], list(range(50)), list(range(49, -1, -1)), [int(v) for v in rng.permutation(3000)],
                  list(range(2999, -1, -1))):
        check(order)
