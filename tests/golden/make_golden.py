"""Regenerate tests/golden/*.npz from the REFERENCE encoder/decoder (oracle/_ref/ref_cdc,
built from /root/reference by `make -C oracle ref`).  Run in the development container
(the reference tree is not available on the GPU box):

    python tests/golden/make_golden.py

Each fixture holds: `rec` (n x 8 int32 canonical input), `max_len`, and either the
reference's output bytes `rempi` + decoded table dump `tables` (int64 dump, see
oracle/tables_format.md) or `ref_failed` = 1 when the reference aborted (REMPI_ERR).
These are data only (inputs and reference outputs); no reference source is stored.
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


def cases():
    yield "kat", S.kat_stream(), 131072, {}
    yield "empty", np.zeros((0, 8), np.int32), 131072, {}
    yield "single_matched", S.permutation_stream([0]), 131072, {}
    yield "only_unmatched", np.array([[3, 2, 0, 0, 0, 0, 0, 5]], np.int32), 131072, {}
    yield "reversed_64", S.permutation_stream(list(range(63, -1, -1))), 131072, {}
    rng = np.random.default_rng(2024)
    for n in [1, 2, 5, 17, 200, 1000, 5000]:
        for mode, J in [("jitter", 0), ("jitter", 1), ("jitter", 4), ("jitter", 32), ("random", 0)]:
            if n >= 1000 and mode == "random" and n > 1000:
                continue
            sets = int(rng.integers(1, 5))
            for mx in ([16, 131072] if n >= 200 else [131072]):
                seed = int(rng.integers(1 << 30))
                recs = S.gen_stream(seed, n, n_sets=sets, n_senders=int(rng.integers(2, 24)), jitter=J,
                                    p_unmatched=0.2, p_group=0.1, mode=mode, neg_index=(n == 200))
                yield f"s{n}_{mode}{J}_t{sets}_m{mx}", recs, mx, {"seed": seed}
    yield "multichunk_small_max", S.gen_stream(7, 3000, n_sets=4, n_senders=16, jitter=8), 64, {}
    yield "unmatched_heavy", S.gen_stream(8, 2000, n_sets=2, n_senders=8, jitter=4, p_unmatched=0.9), 100, {}
    yield "groups_heavy", S.gen_stream(9, 2000, n_sets=3, n_senders=12, jitter=4, p_group=0.6), 64, {}
    yield "sparse_set_ids", S.gen_stream(10, 1500, n_senders=9, jitter=4, set_ids=[0, 7, 128, 255]), 200, {}
    # Synthetic bench workload (gen.h), small rank: the reference on the real trace shape.
    try:
        import rempi_amd as ra

        p = ra.default_gen_params(world_size=64, events_per_rank=30000)
        yield "synthetic_w64_r5_30k", ra.generate_host(p, 5), 131072, {"gen": "world64 rank5 30000"}
        p = ra.default_gen_params(world_size=1024, events_per_rank=20000, jitter=32)
        yield "synthetic_w1024_r1000_j32", ra.generate_host(p, 1000), 4096, {"gen": "world1024 rank1000 j32"}
    except Exception as e:  # noqa: BLE001
        print("skipping synthetic fixtures:", e)
    # Error behaviour: a stream that ends inside a with_next group; a duplicated key.
    trunc = S.permutation_stream([0, 1, 2])
    trunc[-1, 4] = 1
    yield "err_truncated_epoch", trunc, 131072, {}
    dup = S.permutation_stream([0, 1, 2, 3])
    dup[3, 6] = dup[1, 6]  # same (source, clock) twice, not adjacent (no run-length merge)
    yield "err_duplicate_key", dup, 131072, {}


def main():
    if not O.have_ref():
        sys.exit("oracle/_ref/ref_cdc missing: run `make -C oracle ref` in the dev container")
    manifest = {}
    for name, recs, mx, meta in cases():
        d = {"rec": np.ascontiguousarray(recs, np.int32).reshape(-1, 8), "max_len": np.int64(mx)}
        try:
            b, _ = O.ref_encode(recs, mx)
            t, _ = O.ref_decode(b)
            d["rempi"] = np.frombuffer(b, np.uint8)
            d["tables"] = np.frombuffer(t, np.int64)
            d["ref_failed"] = np.int64(0)
        except RuntimeError:
            d["ref_failed"] = np.int64(1)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
        manifest[name] = {"n": int(d["rec"].shape[0]), "max_len": mx, "ref_failed": int(d["ref_failed"]), **meta}
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print(len(manifest), "fixtures")


if __name__ == "__main__":
    main()
