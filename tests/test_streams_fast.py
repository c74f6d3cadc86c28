"""The array-based chunk rule / expected-record builders used for full-size fixtures agree
with the record-by-record ones on small random streams."""
import numpy as np

import cdc_streams as S


def test_fast_builders_match_reference_walk():
    rng = np.random.default_rng(31)
    for t in range(60):
        recs = S.gen_stream(int(rng.integers(1 << 30)), int(rng.integers(0, 1500)), n_sets=int(rng.integers(1, 5)),
                            n_senders=int(rng.integers(1, 20)), jitter=int(rng.choice([0, 4, 32])),
                            p_unmatched=float(rng.choice([0.0, 0.3, 0.8])), p_group=float(rng.choice([0.0, 0.2, 0.6])))
        if t % 3 == 0 and recs.shape[0] > 4:  # consecutive polls of one table split by another table's events
            extra = recs[recs[:, 2] == 0][:3].copy()
            recs = S.canonicalize(np.concatenate([recs[:2], extra, recs[2:], extra]))
        for mx in (1, 7, 100, 131072):
            assert S.chunk_bounds_fast(recs, mx) == S.chunk_bounds(recs, mx)
            np.testing.assert_array_equal(S.expected_table_streams_fast(recs, mx), S.expected_table_streams(recs, mx))
