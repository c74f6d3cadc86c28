"""The C ABI library loads and exports every entry point include/cdcx.h declares (no
device calls here), and the host twin of the synthetic generator behaves."""
import os
import re
import subprocess

import numpy as np

import cdc_streams as S
import oracle_lib as O
import rempi_amd
from rempi_amd import cdcx

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    with open(os.path.join(ROOT, "include", "cdcx.h")) as f:
        text = f.read()
    return sorted(set(re.findall(r"\b(cdcx_[a-z_]+)\s*\(", text)))


def test_header_declares_expected_entry_points():
    syms = declared_symbols()
    for s in ["cdcx_create", "cdcx_encode_stream", "cdcx_encode_chunk", "cdcx_encode_batch_device",
              "cdcx_decode_stream", "cdcx_reconstruct_stream", "cdcx_decode_batch_device"]:
        assert s in syms


def test_library_exports_every_declared_symbol():
    L = rempi_amd.lib()  # loads (fails loudly if libcdcx.so is missing)
    for s in declared_symbols():
        assert hasattr(L, s), s
    nm = subprocess.run(["nm", "-D", "--defined-only", cdcx.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (cdcx_\w+)", nm))
    assert set(declared_symbols()) <= exported
    assert set(cdcx.exported_symbols()) == set(declared_symbols())


def test_generator_host_properties():
    p = rempi_amd.default_gen_params(world_size=64, events_per_rank=20000)
    a = rempi_amd.generate_host(p, 7)
    b = rempi_amd.generate_host(p, 7)
    np.testing.assert_array_equal(a, b)
    assert 19990 <= a.shape[0] <= 20000
    np.testing.assert_array_equal(S.canonicalize(a), a)  # canonical: no run-length merges
    m = a[:, 2] == 1
    assert 0.75 < m.mean() < 0.95
    assert set(np.unique(a[:, 7])) == {0, 1, 2, 3}
    src = a[m, 3]
    assert ((src != 7) & (src >= 0) & (src < 64)).all()
    for s in np.unique(src):  # per-sender clocks strictly increase in clock order
        c = np.sort(a[m][a[m, 3] == s][:, 6])
        assert (np.diff(c) > 0).all()
    # groups never end a table's stream inside with_next, so the oracle accepts it
    O.encode(a, 4096)


def test_generator_small_world():
    p = rempi_amd.default_gen_params(world_size=4, senders=64, sets=4, events_per_rank=500)
    a = rempi_amd.generate_host(p, 0)
    assert set(np.unique(a[a[:, 2] == 1, 3])) <= {1, 2, 3}
    O.encode(a, 131072)
