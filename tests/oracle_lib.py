"""ctypes binding to the CPU oracle (oracle/liboracle_cdc.so) and the reference harness
(oracle/_ref/ref_cdc).  Test infrastructure only: never imported by the product package."""
from __future__ import annotations

import ctypes
import os
import subprocess
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle_cdc.so")
REF_BIN = os.path.join(ROOT, "oracle", "_ref", "ref_cdc")

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "oracle"])
        L = ctypes.CDLL(ORACLE_SO)
        P = ctypes.POINTER
        u8p, i32p, i64p = P(ctypes.c_uint8), P(ctypes.c_int32), P(ctypes.c_int64)
        L.oracle_encode.argtypes = [i32p, ctypes.c_size_t, ctypes.c_int64, P(u8p), P(ctypes.c_size_t), P(ctypes.c_size_t)]
        L.oracle_encode_ex.argtypes = [i32p, ctypes.c_size_t, ctypes.c_int64, ctypes.c_int, P(u8p), P(ctypes.c_size_t),
                                       P(ctypes.c_size_t)]
        L.oracle_decode.argtypes = [u8p, ctypes.c_size_t, P(u8p), P(ctypes.c_size_t)]
        L.oracle_cdc_pairs.argtypes = [i32p, ctypes.c_int64, i32p, i32p, i64p]
        L.oracle_decode_perm.argtypes = [i64p, i64p, ctypes.c_int64, ctypes.c_int64, i32p]
        L.oracle_umap_order.argtypes = [i64p, ctypes.c_int64, i64p]
        L.oracle_umap_order.restype = ctypes.c_int64
        L.oracle_uset_int_order.argtypes = [i32p, ctypes.c_int64, i32p]
        L.oracle_uset_int_order.restype = ctypes.c_int64
        L.oracle_reconstruct.argtypes = [u8p, ctypes.c_size_t, i32p, ctypes.c_size_t, P(i32p), P(ctypes.c_size_t)]
        L.oracle_sorted_keys.argtypes = [i32p, ctypes.c_size_t, ctypes.c_int64, P(i32p), P(ctypes.c_size_t)]
        L.oracle_free.argtypes = [ctypes.c_void_p]
        L.oracle_set_reference_walk.argtypes = [ctypes.c_int]
        L.oracle_set_reference_walk.restype = None
        _lib = L
    return _lib


def _ptr(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


class OracleError(RuntimeError):
    def __init__(self, code):
        super().__init__(f"oracle error {code}")
        self.code = code


def encode(recs: np.ndarray, max_len: int = 131072, rep: bool = False):
    """-> (file bytes, footer offset); rep: the REMPI_ENCODE=7 encoder (epoch lines only)."""
    L = lib()
    r = np.ascontiguousarray(recs, dtype=np.int32).reshape(-1, 8)
    out = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    foff = ctypes.c_size_t()
    rc = L.oracle_encode_ex(_ptr(r, ctypes.c_int32), r.shape[0], max_len, int(rep), ctypes.byref(out), ctypes.byref(n),
                            ctypes.byref(foff))
    if rc:
        raise OracleError(rc)
    data = ctypes.string_at(out, n.value)
    L.oracle_free(out)
    return data, foff.value


def decode(data: bytes) -> bytes:
    """-> int64 table dump (oracle/tables_format.md)."""
    L = lib()
    buf = np.frombuffer(data, dtype=np.uint8).copy()
    out = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    rc = L.oracle_decode(_ptr(buf, ctypes.c_uint8), buf.size, ctypes.byref(out), ctypes.byref(n))
    if rc:
        raise OracleError(rc)
    d = ctypes.string_at(out, n.value)
    L.oracle_free(out)
    return d


def set_reference_walk(on: bool):
    """True: delays longer than the list walk on through the sentinel as in the reference;
    False (default): they are refused, as the device path refuses them."""
    lib().oracle_set_reference_walk(int(on))


def cdc_pairs(c):
    L = lib()
    c = np.ascontiguousarray(c, dtype=np.int32)
    M = c.size
    ids = np.zeros(max(M, 1), np.int32)
    dl = np.zeros(max(M, 1), np.int32)
    P = ctypes.c_int64()
    rc = L.oracle_cdc_pairs(_ptr(c, ctypes.c_int32), M, _ptr(ids, ctypes.c_int32), _ptr(dl, ctypes.c_int32), ctypes.byref(P))
    if rc:
        raise OracleError(rc)
    return ids[: P.value].copy(), dl[: P.value].copy()


def decode_perm(ids, delays, M):
    L = lib()
    a = np.ascontiguousarray(ids, dtype=np.int64)
    d = np.ascontiguousarray(delays, dtype=np.int64)
    perm = np.zeros(max(M, 1), np.int32)
    rc = L.oracle_decode_perm(_ptr(a, ctypes.c_int64), _ptr(d, ctypes.c_int64), a.size, M, _ptr(perm, ctypes.c_int32))
    if rc:
        raise OracleError(rc)
    return perm[:M].copy()


def umap_order(keys):
    L = lib()
    k = np.ascontiguousarray(keys, dtype=np.int64)
    out = np.zeros(max(k.size, 1), np.int64)
    n = L.oracle_umap_order(_ptr(k, ctypes.c_int64), k.size, _ptr(out, ctypes.c_int64))
    return out[:n].copy()


def uset_int_order(keys):
    L = lib()
    k = np.ascontiguousarray(keys, dtype=np.int32)
    out = np.zeros(max(k.size, 1), np.int32)
    n = L.oracle_uset_int_order(_ptr(k, ctypes.c_int32), k.size, _ptr(out, ctypes.c_int32))
    return out[:n].copy()


def sorted_keys(recs, max_len=131072):
    L = lib()
    r = np.ascontiguousarray(recs, dtype=np.int32).reshape(-1, 8)
    out = ctypes.POINTER(ctypes.c_int32)()
    n = ctypes.c_size_t()
    rc = L.oracle_sorted_keys(_ptr(r, ctypes.c_int32), r.shape[0], max_len, ctypes.byref(out), ctypes.byref(n))
    if rc:
        raise OracleError(rc)
    arr = np.ctypeslib.as_array(out, shape=(max(n.value, 1) * 2,))[: 2 * n.value].copy().reshape(-1, 2)
    L.oracle_free(out)
    return arr


def reconstruct(data: bytes, keys: np.ndarray):
    L = lib()
    buf = np.frombuffer(data, dtype=np.uint8).copy()
    k = np.ascontiguousarray(keys, dtype=np.int32).reshape(-1, 2)
    out = ctypes.POINTER(ctypes.c_int32)()
    n = ctypes.c_size_t()
    rc = L.oracle_reconstruct(_ptr(buf, ctypes.c_uint8), buf.size, _ptr(k, ctypes.c_int32), k.shape[0], ctypes.byref(out), ctypes.byref(n))
    if rc:
        raise OracleError(rc)
    arr = np.ctypeslib.as_array(out, shape=(max(n.value, 1) * 8,))[: 8 * n.value].copy().reshape(-1, 8)
    L.oracle_free(out)
    return arr


def parse_tables(dump: bytes):
    """int64 table dump -> list (chunks) of list (tables) of dicts."""
    v = np.frombuffer(dump, dtype=np.int64)
    p = 0
    chunks = []

    def take(n):
        nonlocal p
        a = v[p:p + n]
        p += n
        return a

    def vec():
        n = int(take(1)[0])
        return take(n).copy()

    while p < v.size:
        nt = int(take(1)[0])
        tabs = []
        for _ in range(nt):
            t = {"set_id": int(take(1)[0]), "count": int(take(1)[0])}
            t["epoch_rank"] = vec()
            t["epoch_clock"] = vec()
            t["with_previous"] = vec()
            t["matched_index"] = vec()
            nu = int(take(1)[0])
            t["unmatched"] = take(2 * nu).copy().reshape(-1, 2)
            t["ids"] = vec()
            t["delays"] = vec()
            t["perm"] = vec()
            tabs.append(t)
        chunks.append(tabs)
    return chunks


def have_ref() -> bool:
    return os.path.exists(REF_BIN)


def ref_encode(recs: np.ndarray, max_len: int = 131072, gzip: bool = False, rep: bool = False):
    """Run the reference encoder (oracle/_ref/ref_cdc) -> (bytes, seconds); gzip: REMPI_GZIP=1;
    rep: the REMPI_ENCODE=7 encoder (rempi_encoder_rep, epoch lines only)."""
    with tempfile.TemporaryDirectory() as d:
        inp, outp = os.path.join(d, "in.rec"), os.path.join(d, "out.rempi")
        np.ascontiguousarray(recs, dtype=np.int32).tofile(inp)
        res = subprocess.run([REF_BIN, "encode", inp, outp, str(max_len)] + (["gzip"] if gzip else []) +
                             (["rep"] if rep else []),
                             capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"ref encode failed rc={res.returncode}: {res.stderr[-500:]}")
        secs = float(res.stdout.split()[1])
        with open(outp, "rb") as f:
            return f.read(), secs


def ref_encode_basic(recs: np.ndarray, max_len: int = 131072, gzip: bool = False) -> bytes:
    """Run the reference REMPI_ENCODE=0 encoder (rempi_encoder_basic, via oracle/_ref/ref_cdc
    encode_basic) -> the basic record file: [size_t len][len bytes of 8 x int32] chunks
    (gzip: REMPI_GZIP=1, each chunk payload a zlib stream)."""
    with tempfile.TemporaryDirectory() as d:
        inp, outp = os.path.join(d, "in.rec"), os.path.join(d, "out.basic")
        np.ascontiguousarray(recs, dtype=np.int32).tofile(inp)
        res = subprocess.run([REF_BIN, "encode_basic", inp, outp, str(max_len)] + (["gzip"] if gzip else []),
                             capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"ref encode_basic failed rc={res.returncode}: {res.stderr[-500:]}")
        with open(outp, "rb") as f:
            return f.read()


def parse_basic(data: bytes) -> np.ndarray:
    """Records of a basic record file (rempi_encoder_basic.cpp:238-321 read loop): the chunks'
    8 x int32 events concatenated."""
    out, p = [], 0
    while p < len(data):
        n = int(np.frombuffer(data[p:p + 8], np.uint64)[0])
        p += 8
        out.append(np.frombuffer(data[p:p + n], np.int32).reshape(-1, 8))
        p += n
    return np.concatenate(out) if out else np.zeros((0, 8), np.int32)


def ref_decode(data: bytes, gzip: bool = False):
    with tempfile.TemporaryDirectory() as d:
        inp, outp = os.path.join(d, "in.rempi"), os.path.join(d, "out.tables")
        with open(inp, "wb") as f:
            f.write(data)
        res = subprocess.run([REF_BIN, "decode", inp, outp] + (["gzip"] if gzip else []), capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"ref decode failed rc={res.returncode}: {res.stderr[-500:]}")
        secs = float(res.stdout.split()[1])
        with open(outp, "rb") as f:
            return f.read(), secs
