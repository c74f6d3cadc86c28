"""Config 1 of BASELINE.json as fixtures: the event streams ReMPI records for
`rempi_test_units matching` on 4 ranks (test/rempi/rempi_test_units.c:381-542, driven by
:1165-1172), encoded and decoded by the REFERENCE (oracle/_ref/ref_cdc).

    python tests/golden/make_config1_golden.py

The test program cannot run here (no MPI launcher with PMPI interposition, no CLMPI), so the
streams are an emulation of what rempi_recorder::record_mf (rempi_recorder.cpp:507-694) pushes
for it:
  * ranks 1..3 send NUM_TEST_MSG = 4 messages each to rank 0 in each of the 8 phases (one per
    matching function id, :104-107: Test, Testany, Testsome, Testall, Wait, Waitany, Waitsome,
    Waitall) with MPI_ANY_SOURCE / MPI_ANY_TAG receives, a barrier after each phase;
  * rank 0 records one test event per matching-function call: unmatched polls
    (flag 0, run-length merged by rempi_event_list::push) for the Test* functions, matched
    events {count 1, flag 1, source, with_next, request index, clock, matching set id}, the
    events of one Testsome/Testall/Waitsome/Waitall call chained by with_next;
  * clocks are Lamport clocks as rempi_clock.cpp keeps them: start 10, +1 per send, the
    message carries the sender's clock, a barrier lifts every clock to the maximum + 3;
  * every phase is its own matching set (the request manager gives each call site an id).
Ranks 1..3 call no matching function, so their streams are empty (a rank file with only the
footer).  The seed varies the arrival interleaving; several seeds are kept.  With
REMPI_MAX = 8 the 96 matched events span several chunks as well.
Fixtures have the layout of make_golden.py and are added to manifest.json.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import cdc_streams as S  # noqa: E402
import oracle_lib as O  # noqa: E402

NUM_TEST_MSG = 4
PHASES = ["Test", "Testany", "Testsome", "Testall", "Wait", "Waitany", "Waitsome", "Waitall"]


def rank0_stream(seed: int, n_ranks: int = 4) -> np.ndarray:
    rng = np.random.default_rng(seed)
    senders = list(range(1, n_ranks))
    ns = len(senders)
    clock = {r: 10 for r in range(n_ranks)}
    recs = []

    def poll(set_id):
        recs.append([1, 2, 0, 0, 0, 0, 0, set_id])

    def matched(group, set_id):
        for k, (src, clk, idx) in enumerate(group):
            recs.append([1, 2, 1, src, 1 if k + 1 < len(group) else 0, idx, clk, set_id])
            clock[0] = max(clock[0], clk) + 1

    for set_id, phase in enumerate(PHASES):
        # messages in flight: per sender in send order, interleaved at random on arrival
        queues = {s: [] for s in senders}
        for s in senders:
            for _ in range(NUM_TEST_MSG):
                clock[s] += 1
                queues[s].append(clock[s])
        arrival = []
        left = {s: list(q) for s, q in queues.items()}
        while any(left.values()):
            s = int(rng.choice([x for x in senders if left[x]]))
            arrival.append((s, left[s].pop(0)))
        req = 0  # round-robin request index of Test / Wait
        total = ns * NUM_TEST_MSG
        done = 0
        while done < total:
            if phase.startswith("Test"):
                for _ in range(int(rng.integers(0, 4))):
                    poll(set_id)
            if phase in ("Test", "Wait"):
                s, c = arrival.pop(0)
                matched([(s, c, 0)], set_id)  # single-request function: matched_index = 0
                req = (req + 1) % ns
                done += 1
            elif phase in ("Testany", "Waitany"):
                s, c = arrival.pop(0)
                matched([(s, c, int(rng.integers(ns)))], set_id)
                done += 1
            elif phase in ("Testsome", "Waitsome"):
                k = min(int(rng.integers(1, ns + 1)), len(arrival))
                idx = rng.permutation(ns)[:k]
                matched([(arrival[i][0], arrival[i][1], int(idx[i])) for i in range(k)], set_id)
                del arrival[:k]
                done += k
            else:  # Testall / Waitall: all num_sender requests complete in one call
                matched([(arrival[i][0], arrival[i][1], i) for i in range(ns)], set_id)
                del arrival[:ns]
                done += ns
        top = max(clock.values()) + 3  # barrier: collective clock synchronisation
        for r in clock:
            clock[r] = top
    return S.canonicalize(np.array(recs, np.int32))


def cases():
    for seed in (1, 2, 3):
        yield f"config1_matching_r0_seed{seed}", rank0_stream(seed), 131072, {"config": 1, "seed": seed}
    yield "config1_matching_r0_seed1_max8", rank0_stream(1), 8, {"config": 1, "seed": 1}
    for r in (1, 2, 3):
        yield f"config1_matching_r{r}", np.zeros((0, 8), np.int32), 131072, {"config": 1, "sender_rank": r}


def main():
    if not O.have_ref():
        sys.exit("oracle/_ref/ref_cdc missing: run `make -C oracle ref` in the dev container")
    with open(os.path.join(HERE, "manifest.json")) as f:
        manifest = json.load(f)
    for name, recs, mx, meta in cases():
        b, _ = O.ref_encode(recs, mx)
        t, _ = O.ref_decode(b)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), rec=np.ascontiguousarray(recs, np.int32).reshape(-1, 8),
                            max_len=np.int64(mx), rempi=np.frombuffer(b, np.uint8), tables=np.frombuffer(t, np.int64),
                            ref_failed=np.int64(0))
        manifest[name] = {"n": int(recs.shape[0]), "max_len": mx, "ref_failed": 0, **meta}
        print(f"{name}: {recs.shape[0]} records -> {len(b)} B")
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
