"""The drop-in shim (oracle/shim/rempi_encoder_cdcx.h) under the reference's own loops.

oracle/_ref/shim_cdc is the reference's record loop (rempi_io_thread.cpp:56-97:
extract_encoder_input_format_chunk -> encode -> write_record_file -> close_record_file) and
replay read loop (rempi_encoder_cdc.cpp:851-930: read_record_file -> decode) compiled from
the unmodified reference sources, with rempi_encoder_cdcx -- encode() = cdcx_encode_chunk,
decode() = cdcx_decode_chunk -- in place of rempi_encoder_cdc.  Its files must equal the
reference-written golden bytes and its test tables the reference's decode()."""
import os
import subprocess

import numpy as np
import pytest

import golden_util as G

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "oracle", "_ref", "shim_cdc")
OK_NAMES = [n for n in G.names() if not G.load(n)["ref_failed"]]

pytestmark = pytest.mark.gpu


def run_batch(tmp_path, lines):
    lst = tmp_path / "batch.txt"
    lst.write_text("\n".join(lines) + "\n")
    res = subprocess.run([SHIM, "batch", str(lst)], capture_output=True, text=True, timeout=600)
    assert res.returncode == 0, (res.returncode, res.stdout[-500:], res.stderr[-2000:])
    return res


@pytest.fixture(scope="module")
def have_shim():
    if not os.path.exists(SHIM):
        pytest.fail("oracle/_ref/shim_cdc is not built (make -C oracle shim; needs /root/reference)")


def test_record_loop_writes_reference_files(tmp_path, have_shim):
    lines = []
    for n in OK_NAMES:
        d = G.load(n)
        np.ascontiguousarray(d["rec"], dtype=np.int32).tofile(tmp_path / f"{n}.rec")
        lines.append(f"encode {tmp_path / (n + '.rec')} {tmp_path / (n + '.rempi')} {d['max_len']}")
    run_batch(tmp_path, lines)
    bad = [n for n in OK_NAMES if (tmp_path / f"{n}.rempi").read_bytes() != G.load(n)["rempi"]]
    assert not bad, bad


def test_replay_loop_fills_reference_tables(tmp_path, have_shim):
    lines = []
    for n in OK_NAMES:
        (tmp_path / f"{n}.rempi").write_bytes(G.load(n)["rempi"])
        lines.append(f"decode {tmp_path / (n + '.rempi')} {tmp_path / (n + '.tables')}")
    run_batch(tmp_path, lines)
    bad = [n for n in OK_NAMES if (tmp_path / f"{n}.tables").read_bytes() != G.load(n)["tables"]]
    assert not bad, bad


def test_gzip_files_through_reference_zlib_stage(tmp_path, have_shim):
    """REMPI_GZIP=1: the shim leaves write_record_file / read_record_file's zlib stage to the
    reference, so the gzip fixtures come out byte-identical as well."""
    lines, names = [], G.gzip_names()
    for n in names:
        d = G.load_gzip(n)
        np.ascontiguousarray(d["rec"], dtype=np.int32).tofile(tmp_path / f"{n}.rec")
        (tmp_path / f"{n}.in.rempi").write_bytes(d["rempi_gz"])
        lines.append(f"encode {tmp_path / (n + '.rec')} {tmp_path / (n + '.rempi')} {d['max_len']} gzip")
        lines.append(f"decode {tmp_path / (n + '.in.rempi')} {tmp_path / (n + '.tables')} gzip")
    run_batch(tmp_path, lines)
    for n in names:
        d = G.load_gzip(n)
        assert (tmp_path / f"{n}.rempi").read_bytes() == d["rempi_gz"], n
        assert (tmp_path / f"{n}.tables").read_bytes() == d["tables"], n
