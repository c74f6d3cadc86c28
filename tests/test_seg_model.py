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
    stats = {}
    got = SM.rebuild(ids, dl, len(order), stats)
    if got is not None:
        assert got == [int(v) for v in want]
    return got is not None, SM.nseg(len(ids)), stats.get("reruns", 0)


@pytest.mark.parametrize("reach,expect_pass", [(6, True), (12, True), (40, None), (150, None), (2000, None)])
def test_segments_vs_sequential_replay(reach, expect_pass):
    rng = np.random.default_rng(17 + reach)
    passed = multi = 0
    for t in range(6):
        n = int(rng.integers(5000, 12000))
        ok, ns, _ = check(moved(n, rng, n, reach))
        passed += ok
        multi += ns > 1
    assert multi == 6  # (several segments each: the check between them ran)
    if expect_pass:
        assert passed == 6


def test_rerun_on_bench_trace():
    """Ranks 317 and 446 of the bench workload (400 K events) each have a table with a segment
    whose replay gives another state than its predecessor ends in (rank 317 with segments of 1024
    pairs, rank 446 with 2048); run again from that state the table comes out as the sequential
    replay's.  (tests/test_gpu_parity.py runs the same traces on the device.)"""
    import rempi_amd

    p = rempi_amd.default_gen_params(world_size=1024, events_per_rank=400_000)
    reruns = 0
    for rank in (317, 446):
        data, _ = O.encode(rempi_amd.generate_host(p, rank), 131072)
        for chunk in O.parse_tables(O.decode(data)):
            for t in chunk:
                stats = {}
                got = SM.rebuild(t["ids"], t["delays"], t["count"], stats)
                assert got is not None and got == [int(v) for v in t["perm"]]
                reruns += stats.get("reruns", 0)
    assert reruns >= 1


def test_small_and_degenerate():
    rng = np.random.default_rng(9)
    for order in ([], [0], [1, 0], list(range(50)), list(range(49, -1, -1)), [int(v) for v in rng.permutation(3000)],
                  list(range(2999, -1, -1))):
        check(order)
