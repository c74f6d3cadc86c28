"""ctypes binding of libcdcx.so (include/cdcx.h).

This is plumbing for tests and bench.py: every codec byte is produced by the HIP kernels
behind the C ABI.  Loading fails loudly when the library is missing -- there is no CPU
fallback on the product path.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# CDCX_LIB: another in-tree build of the same library (A/B timing of kernel variants)
LIB_PATH = os.path.join(HERE, os.environ.get("CDCX_LIB", "libcdcx.so"))

CDCX_OK = 0
ERRORS = {
    1: "CDCX_ERR_ARG",
    2: "CDCX_ERR_TRUNCATED_EPOCH",
    3: "CDCX_ERR_CLOCK_ORDER",
    4: "CDCX_ERR_CORRUPT",
    5: "CDCX_ERR_HIP",
    6: "CDCX_ERR_LIMIT",
    7: "CDCX_ERR_NOMEM",
}


class CdcxError(RuntimeError):
    def __init__(self, code: int, msg: str = ""):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class _Opts(ctypes.Structure):
    _fields_ = [("max_event_length", ctypes.c_int64), ("gzip", ctypes.c_int32), ("device", ctypes.c_int32),
                ("encode", ctypes.c_int32), ("pad", ctypes.c_int32), ("reserved", ctypes.c_int64 * 3)]


class GenParams(ctypes.Structure):
    _fields_ = [("world_size", ctypes.c_int32), ("senders", ctypes.c_int32), ("sets", ctypes.c_int32),
                ("jitter", ctypes.c_int32), ("events_per_rank", ctypes.c_int64), ("seed_salt", ctypes.c_uint64)]


P = ctypes.POINTER
_u8p, _i32p, _i64p, _vp = P(ctypes.c_uint8), P(ctypes.c_int32), P(ctypes.c_int64), ctypes.c_void_p


class ReplayStats(ctypes.Structure):
    _fields_ = [("files", ctypes.c_int64), ("file_bytes", ctypes.c_int64), ("chunks", ctypes.c_int64),
                ("units", ctypes.c_int64), ("records", ctypes.c_int64), ("batches", ctypes.c_int64),
                ("dump_bytes", ctypes.c_int64), ("seconds", ctypes.c_double), ("read_s", ctypes.c_double),
                ("device_s", ctypes.c_double), ("dump_s", ctypes.c_double), ("sink_s", ctypes.c_double)]


class Table(ctypes.Structure):
    """cdcx_table: one decoded matching-set table of a chunk (flat arrays)."""
    _fields_ = [("set_id", ctypes.c_int32), ("count", ctypes.c_int32),
                ("n_epoch", ctypes.c_size_t), ("epoch_rank", P(ctypes.c_uint64)), ("epoch_clock", P(ctypes.c_uint64)),
                ("n_with_previous", ctypes.c_size_t), ("with_previous", P(ctypes.c_uint64)),
                ("n_matched_index", ctypes.c_size_t), ("matched_index", P(ctypes.c_uint64)),
                ("n_unmatched", ctypes.c_size_t), ("unmatched_id", P(ctypes.c_uint64)),
                ("unmatched_count", P(ctypes.c_uint64)),
                ("n_pairs", ctypes.c_size_t), ("ids", P(ctypes.c_uint64)), ("delays", P(ctypes.c_uint64)),
                ("perm", P(ctypes.c_int32))]


class Tables(ctypes.Structure):
    _fields_ = [("n_tables", ctypes.c_size_t), ("tables", P(Table))]


_REPLAY_SINK = ctypes.CFUNCTYPE(ctypes.c_int, _vp, ctypes.c_int32, _i64p, ctypes.c_size_t)

_REPLAY_TABLE_SINK = ctypes.CFUNCTYPE(ctypes.c_int, _vp, ctypes.c_int32, ctypes.c_size_t, P(Tables))


class FooterInfo(ctypes.Structure):
    _fields_ = [("n_ranks", ctypes.c_size_t), ("ranks", _i32p), ("n_ids", ctypes.c_size_t),
                ("msg_ids", P(ctypes.c_uint64)), ("set_ids", _i32p)]


_REPLAY_FOOTER_SINK = ctypes.CFUNCTYPE(ctypes.c_int, _vp, ctypes.c_int32, P(FooterInfo))

_SIGNATURES = {
    "cdcx_create": ([P(_Opts)], _vp),
    "cdcx_destroy": ([_vp], None),
    "cdcx_last_error": ([_vp], ctypes.c_char_p),
    "cdcx_free": ([_vp], None),
    "cdcx_kernel_count": ([], ctypes.c_int),
    "cdcx_kernel_name": ([ctypes.c_int], ctypes.c_char_p),
    "cdcx_encode_stream": ([_vp, _i32p, ctypes.c_size_t, P(_u8p), P(ctypes.c_size_t)], ctypes.c_int),
    "cdcx_gzip_file": ([_u8p, ctypes.c_size_t, P(_u8p), P(ctypes.c_size_t)], ctypes.c_int),
    "cdcx_gunzip_file": ([_u8p, ctypes.c_size_t, P(_u8p), P(ctypes.c_size_t)], ctypes.c_int),
    "cdcx_transcode_basic": ([_vp, ctypes.c_size_t, P(_u8p), P(ctypes.c_size_t), P(_u8p), P(ctypes.c_size_t)], ctypes.c_int),
    "cdcx_encode_chunk": ([_vp, _i32p, ctypes.c_size_t, P(_u8p), P(ctypes.c_size_t), P(_i32p), P(ctypes.c_size_t)], ctypes.c_int),
    "cdcx_encode_batch_device": ([_vp, ctypes.c_int32, _vp, _i64p, P(_vp), _i64p, _i64p, _vp], ctypes.c_int),
    "cdcx_batch_sorted_keys": ([_vp, P(_vp), _i64p], ctypes.c_int),
    "cdcx_decode_stream": ([_vp, _u8p, ctypes.c_size_t, P(_u8p), P(ctypes.c_size_t)], ctypes.c_int),
    "cdcx_reconstruct_stream": ([_vp, _u8p, ctypes.c_size_t, _i32p, ctypes.c_size_t, P(_i32p), P(ctypes.c_size_t)], ctypes.c_int),
    "cdcx_decode_chunk": ([_vp, _u8p, ctypes.c_size_t, P(Tables)], ctypes.c_int),
    "cdcx_reconstruct_chunk": ([_vp, _u8p, ctypes.c_size_t, _i32p, ctypes.c_size_t, P(_i32p), P(ctypes.c_size_t)], ctypes.c_int),
    "cdcx_footer": ([_i32p, ctypes.c_size_t, _u8p, P(ctypes.c_size_t)], ctypes.c_int),
    "cdcx_footer_ex": ([_i32p, ctypes.c_size_t, P(ctypes.c_uint64), _i32p, ctypes.c_size_t, _u8p, P(ctypes.c_size_t)],
                       ctypes.c_int),
    "cdcx_set_matching_set_id_map": ([_vp, P(ctypes.c_uint64), _i32p, ctypes.c_size_t], ctypes.c_int),
    "cdcx_read_footer": ([_u8p, ctypes.c_size_t, P(P(FooterInfo))], ctypes.c_int),
    "cdcx_replay_decode_tables_ex": ([P(_vp), ctypes.c_int32, ctypes.c_int32, P(ctypes.c_char_p), ctypes.c_int64,
                                      _REPLAY_TABLE_SINK, _REPLAY_FOOTER_SINK, _vp, P(ReplayStats)], ctypes.c_int),
    "cdcx_decode_batch_device": ([_vp, ctypes.c_int32, _vp, _i64p, _i64p, _vp, ctypes.c_int64, P(_vp), _i64p, P(_vp), _vp], ctypes.c_int),
    "cdcx_decode_chunk_perm_static": ([_vp, _vp, ctypes.c_size_t, _vp, ctypes.c_size_t, _i64p, _vp], ctypes.c_int),
    "cdcx_decode_rank_offsets": ([_vp, ctypes.c_int32, _i64p, _i64p], ctypes.c_int),
    "cdcx_verify_roundtrip_device": ([_vp, _vp, _i64p, _vp], ctypes.c_int),
    "cdcx_replay_decode_files": ([P(_vp), ctypes.c_int32, ctypes.c_int32, P(ctypes.c_char_p), ctypes.c_int64,
                                  _REPLAY_SINK, _vp, P(ReplayStats)], ctypes.c_int),
    "cdcx_replay_decode_tables": ([P(_vp), ctypes.c_int32, ctypes.c_int32, P(ctypes.c_char_p), ctypes.c_int64,
                                   _REPLAY_TABLE_SINK, _vp, P(ReplayStats)], ctypes.c_int),
    "cdcx_generate_device": ([_vp, P(GenParams), ctypes.c_int32, ctypes.c_int32, P(_vp), _i64p, _vp], ctypes.c_int),
    "cdcx_generate_host": ([P(GenParams), ctypes.c_int32, P(_i32p), P(ctypes.c_size_t)], ctypes.c_int),
    "cdcx_set_profiling": ([_vp, ctypes.c_int], ctypes.c_int),
    "cdcx_kernel_times": ([_vp, P(ctypes.c_double), _i64p, ctypes.c_int], ctypes.c_int),
    "cdcx_reset_kernel_times": ([_vp], ctypes.c_int),
    "cdcx_chain_stats": ([_vp, _i64p, ctypes.c_int], ctypes.c_int),
    "cdcx_chain_tiers": ([_vp, _i64p], ctypes.c_int),
    "cdcx_decode_tiers": ([_vp, _i64p], ctypes.c_int),
    "cdcx_encode_totals": ([_vp, _i64p], ctypes.c_int),
}

_lib = None


def lib() -> ctypes.CDLL:
    """Load libcdcx.so; raises if it is absent (no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = ctypes.CDLL(LIB_PATH)
        for name, (args, res) in _SIGNATURES.items():
            if "CDCX_LIB" in os.environ and not hasattr(L, name):
                continue  # (an older build in an A/B run: its diagnostics calls then fail when used)
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        _lib = L
    return _lib


def exported_symbols():
    return list(_SIGNATURES)


def _ptr(a, t):
    return a.ctypes.data_as(P(t))


def default_gen_params(world_size=1024, senders=64, sets=4, jitter=8, events_per_rank=10_000_000, seed_salt=0):
    return GenParams(world_size, senders, sets, jitter, events_per_rank, seed_salt)


def generate_host(params: GenParams, rank: int) -> np.ndarray:
    """Synthetic trace of one rank (host twin of the device generator)."""
    L = lib()
    out = _i32p()
    n = ctypes.c_size_t()
    rc = L.cdcx_generate_host(ctypes.byref(params), rank, ctypes.byref(out), ctypes.byref(n))
    if rc:
        raise CdcxError(rc, "generate_host")
    arr = np.ctypeslib.as_array(out, shape=(max(n.value, 1) * 8,))[: 8 * n.value].copy().reshape(-1, 8)
    L.cdcx_free(out)
    return arr


def _zlib_stage(fn, data: bytes) -> bytes:
    L = lib()
    buf = np.frombuffer(bytes(data), dtype=np.uint8) if data else np.zeros(1, np.uint8)
    out = _u8p()
    n = ctypes.c_size_t()
    rc = fn(buf.ctypes.data_as(_u8p), len(data), ctypes.byref(out), ctypes.byref(n))
    if rc != 0:
        raise CdcxError(rc, "zlib stage")
    res = ctypes.string_at(out, n.value)
    L.cdcx_free(out)
    return res


def gzip_file(data: bytes) -> bytes:
    """A plain CDC rank file -> its REMPI_GZIP=1 form (cdcx_gzip_file; host only, no GPU)."""
    return _zlib_stage(lib().cdcx_gzip_file, data)


def gunzip_file(data: bytes) -> bytes:
    """A REMPI_GZIP=1 CDC rank file -> the plain one (cdcx_gunzip_file; host only, no GPU)."""
    return _zlib_stage(lib().cdcx_gunzip_file, data)


def footer(epoch_ranks, msg_ids=None, set_ids=None) -> bytes:
    """write_footer's bytes for the epoch ranks inserted in this order and, optionally, the
    matching-set-id map registered in this order (cdcx_footer / cdcx_footer_ex; host only)."""
    L = lib()
    r = np.ascontiguousarray(epoch_ranks, dtype=np.int32)
    n = ctypes.c_size_t(0)
    if msg_ids is None:
        call = lambda out: L.cdcx_footer(_ptr(r, ctypes.c_int32), r.size, out, ctypes.byref(n))  # noqa: E731
    else:
        m = np.ascontiguousarray(msg_ids, dtype=np.uint64)
        q = np.ascontiguousarray(set_ids, dtype=np.int32)
        assert m.size == q.size
        call = lambda out: L.cdcx_footer_ex(_ptr(r, ctypes.c_int32), r.size, _ptr(m, ctypes.c_uint64),  # noqa: E731
                                            _ptr(q, ctypes.c_int32), m.size, out, ctypes.byref(n))
    rc = call(None)
    if rc:
        raise CdcxError(rc, "footer size")
    out = np.zeros(n.value, np.uint8)
    rc = call(_ptr(out, ctypes.c_uint8))
    if rc:
        raise CdcxError(rc, "footer")
    return out[: n.value].tobytes()


def _footer_dict(fi) -> dict:
    def arr(ptr, n, dt):
        return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dt).copy() if n else np.zeros(0, dt)

    return {"ranks": arr(fi.ranks, fi.n_ranks, np.int32), "msg_ids": arr(fi.msg_ids, fi.n_ids, np.uint64),
            "set_ids": arr(fi.set_ids, fi.n_ids, np.int32)}


def read_footer(data: bytes) -> dict:
    """read_footer of a rank file image: {"ranks", "msg_ids", "set_ids"} in file order
    (cdcx_read_footer; host only)."""
    L = lib()
    buf = np.frombuffer(data, dtype=np.uint8)
    out = P(FooterInfo)()
    rc = L.cdcx_read_footer(_ptr(buf, ctypes.c_uint8), buf.size, ctypes.byref(out))
    if rc:
        raise CdcxError(rc, "read_footer")
    d = _footer_dict(out.contents)
    L.cdcx_free(out)
    return d


class Context:
    """One codec context on one HIP device (cdcx_create / cdcx_destroy)."""

    def __init__(self, max_event_length: int = 131072, device: int = 0, gzip: int = 0, encode: int = 4):
        """gzip=1 is REMPI_GZIP=1: the host-buffer calls apply the zlib stage on the host.
        encode is REMPI_ENCODE: 4 = CDC, 7 = rep (epoch lines only)."""
        L = lib()
        opts = _Opts(max_event_length, gzip, device, encode, 0, (ctypes.c_int64 * 3)())
        self._c = L.cdcx_create(ctypes.byref(opts))
        if not self._c:
            raise CdcxError(5, f"cdcx_create failed (device {device})")
        self.max_event_length = max_event_length

    def set_matching_set_id_map(self, msg_ids=(), set_ids=()):
        """rempi_reqmg_set_matching_set_id_map: entries the files written by encode_stream /
        transcode_basic then carry in their footer; no entries = forget the map."""
        m = np.ascontiguousarray(msg_ids, dtype=np.uint64)
        q = np.ascontiguousarray(set_ids, dtype=np.int32)
        assert m.size == q.size
        self._check(lib().cdcx_set_matching_set_id_map(self._c, _ptr(m, ctypes.c_uint64), _ptr(q, ctypes.c_int32), m.size),
                    "set_matching_set_id_map")

    def close(self):
        if getattr(self, "_c", None):
            lib().cdcx_destroy(self._c)
            self._c = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != CDCX_OK:
            raise CdcxError(rc, f"{what}: {lib().cdcx_last_error(self._c).decode(errors='replace')}")

    # -- host-buffer entry points ------------------------------------------------------
    def encode_stream(self, recs: np.ndarray) -> bytes:
        L = lib()
        r = np.ascontiguousarray(recs, dtype=np.int32).reshape(-1, 8)
        out = _u8p()
        n = ctypes.c_size_t()
        self._check(L.cdcx_encode_stream(self._c, _ptr(r, ctypes.c_int32), r.shape[0], ctypes.byref(out), ctypes.byref(n)),
                    "encode_stream")
        data = ctypes.string_at(out, n.value)
        L.cdcx_free(out)
        return data

    def transcode_basic(self, files):
        """REMPI_ENCODE=0 record files (bytes each, one rank per file) -> their CDC rank files,
        encoded as one device batch (cdcx_transcode_basic)."""
        L = lib()
        files = [bytes(f) for f in files]
        n = len(files)
        bufs = [np.frombuffer(f, dtype=np.uint8) if f else np.zeros(1, np.uint8) for f in files]
        ptrs = (_u8p * max(n, 1))(*[b.ctypes.data_as(_u8p) for b in bufs])
        lens = (ctypes.c_size_t * max(n, 1))(*[len(f) for f in files])
        outs = (_u8p * max(n, 1))()
        olens = (ctypes.c_size_t * max(n, 1))()
        self._check(L.cdcx_transcode_basic(self._c, n, ptrs, lens, outs, olens), "transcode_basic")
        res = []
        for i in range(n):
            res.append(ctypes.string_at(outs[i], olens[i]))
            L.cdcx_free(outs[i])
        return res

    def encode_chunk(self, recs: np.ndarray):
        L = lib()
        r = np.ascontiguousarray(recs, dtype=np.int32).reshape(-1, 8)
        out = _u8p()
        n = ctypes.c_size_t()
        er = _i32p()
        ne = ctypes.c_size_t()
        self._check(L.cdcx_encode_chunk(self._c, _ptr(r, ctypes.c_int32), r.shape[0], ctypes.byref(out), ctypes.byref(n),
                                        ctypes.byref(er), ctypes.byref(ne)), "encode_chunk")
        data = ctypes.string_at(out, n.value)
        ranks = np.ctypeslib.as_array(er, shape=(max(ne.value, 1),))[: ne.value].copy()
        L.cdcx_free(out)
        L.cdcx_free(er)
        return data, ranks

    def decode_stream(self, data: bytes) -> bytes:
        L = lib()
        buf = np.frombuffer(data, dtype=np.uint8).copy()
        out = _u8p()
        n = ctypes.c_size_t()
        self._check(L.cdcx_decode_stream(self._c, _ptr(buf, ctypes.c_uint8), buf.size, ctypes.byref(out), ctypes.byref(n)),
                    "decode_stream")
        d = ctypes.string_at(out, n.value)
        L.cdcx_free(out)
        return d

    def decode_chunk(self, payload: bytes):
        """One chunk payload -> list of dicts (ascending set id) with the decoded table fields
        (cdcx_decode_chunk)."""
        L = lib()
        buf = np.frombuffer(bytes(payload), dtype=np.uint8).copy() if payload else np.zeros(1, np.uint8)
        t = Tables()
        self._check(L.cdcx_decode_chunk(self._c, _ptr(buf, ctypes.c_uint8), len(payload), ctypes.byref(t)), "decode_chunk")

        out = [_table_dict(t.tables[i]) for i in range(t.n_tables)]
        L.cdcx_free(t.tables)
        return out

    def reconstruct_chunk(self, payload: bytes, keys: np.ndarray) -> np.ndarray:
        L = lib()
        buf = np.frombuffer(bytes(payload), dtype=np.uint8).copy()
        k = np.ascontiguousarray(keys, dtype=np.int32).reshape(-1, 2)
        out = _i32p()
        n = ctypes.c_size_t()
        self._check(L.cdcx_reconstruct_chunk(self._c, _ptr(buf, ctypes.c_uint8), buf.size, _ptr(k, ctypes.c_int32),
                                             k.shape[0], ctypes.byref(out), ctypes.byref(n)), "reconstruct_chunk")
        arr = np.ctypeslib.as_array(out, shape=(max(n.value, 1) * 8,))[: 8 * n.value].copy().reshape(-1, 8)
        L.cdcx_free(out)
        return arr

    def reconstruct_stream(self, data: bytes, keys: np.ndarray) -> np.ndarray:
        L = lib()
        buf = np.frombuffer(data, dtype=np.uint8).copy()
        k = np.ascontiguousarray(keys, dtype=np.int32).reshape(-1, 2)
        out = _i32p()
        n = ctypes.c_size_t()
        self._check(L.cdcx_reconstruct_stream(self._c, _ptr(buf, ctypes.c_uint8), buf.size, _ptr(k, ctypes.c_int32),
                                              k.shape[0], ctypes.byref(out), ctypes.byref(n)), "reconstruct_stream")
        arr = np.ctypeslib.as_array(out, shape=(max(n.value, 1) * 8,))[: 8 * n.value].copy().reshape(-1, 8)
        L.cdcx_free(out)
        return arr

    # -- device-resident batch entry points (pointers are device addresses) ----------------
    def generate_device(self, params: GenParams, first_rank: int, n_ranks: int, stream=None):
        """-> (device pointer to records, rec_off numpy[n_ranks+1])"""
        L = lib()
        d = _vp()
        off = np.zeros(n_ranks + 1, np.int64)
        self._check(L.cdcx_generate_device(self._c, ctypes.byref(params), first_rank, n_ranks, ctypes.byref(d),
                                           _ptr(off, ctypes.c_int64), stream), "generate_device")
        return d.value, off

    def encode_batch_device(self, d_rec: int, rec_off: np.ndarray, stream=None):
        """-> (device pointer to output, out_off[n], out_len[n])"""
        L = lib()
        n = rec_off.size - 1
        ro = np.ascontiguousarray(rec_off, dtype=np.int64)
        d = _vp()
        oo = np.zeros(n, np.int64)
        ol = np.zeros(n, np.int64)
        self._check(L.cdcx_encode_batch_device(self._c, n, d_rec, _ptr(ro, ctypes.c_int64), ctypes.byref(d),
                                               _ptr(oo, ctypes.c_int64), _ptr(ol, ctypes.c_int64), stream),
                    "encode_batch_device")
        return d.value, oo, ol

    def batch_sorted_keys(self):
        L = lib()
        d = _vp()
        n = ctypes.c_int64()
        self._check(L.cdcx_batch_sorted_keys(self._c, ctypes.byref(d), ctypes.byref(n)), "batch_sorted_keys")
        return d.value, n.value

    def decode_batch_device(self, d_in: int, in_off: np.ndarray, in_len: np.ndarray, d_keys=None, n_keys=0, stream=None):
        """-> (device records pointer, n records, device perm pointer)"""
        L = lib()
        n = in_off.size
        oo = np.ascontiguousarray(in_off, dtype=np.int64)
        ol = np.ascontiguousarray(in_len, dtype=np.int64)
        dr = _vp()
        nr = ctypes.c_int64()
        dp = _vp()
        self._check(L.cdcx_decode_batch_device(self._c, n, d_in, _ptr(oo, ctypes.c_int64), _ptr(ol, ctypes.c_int64),
                                               d_keys, n_keys, ctypes.byref(dr), ctypes.byref(nr), ctypes.byref(dp),
                                               stream), "decode_batch_device")
        return dr.value, nr.value, dp.value

    def decode_chunk_perm_static(self, d_payload: int, nbytes: int, d_perm: int, perm_capacity: int, stream=None) -> int:
        """cdcx_decode_chunk_perm_static: device payload -> device perm; returns the entries written."""
        n = ctypes.c_int64(-1)
        self._check(lib().cdcx_decode_chunk_perm_static(self._c, d_payload, nbytes, d_perm, perm_capacity, ctypes.byref(n),
                                                        stream), "decode_chunk_perm_static")
        return n.value

    def decode_rank_offsets(self, n_ranks: int):
        """After decode_batch_device: (record offsets, perm offsets) of each rank, n_ranks + 1 each."""
        ro = np.zeros(n_ranks + 1, np.int64)
        po = np.zeros(n_ranks + 1, np.int64)
        self._check(lib().cdcx_decode_rank_offsets(self._c, n_ranks, _ptr(ro, ctypes.c_int64), _ptr(po, ctypes.c_int64)),
                    "decode_rank_offsets")
        return ro, po

    def verify_roundtrip_device(self, d_rec: int, stream=None) -> int:
        """After encode_batch_device(d_rec) + decode_batch_device of its files and keys: the
        number of decoded records that differ from their input record (device-side check)."""
        n = ctypes.c_int64(-1)
        self._check(lib().cdcx_verify_roundtrip_device(self._c, d_rec, ctypes.byref(n), stream), "verify_roundtrip_device")
        return n.value

    # -- profiling -----------------------------------------------------------------------
    def set_profiling(self, on: bool):
        self._check(lib().cdcx_set_profiling(self._c, 1 if on else 0), "set_profiling")

    def kernel_times(self):
        L = lib()
        k = L.cdcx_kernel_count()
        ms = (ctypes.c_double * k)()
        ln = (ctypes.c_int64 * k)()
        self._check(L.cdcx_kernel_times(self._c, ms, ln, k), "kernel_times")
        return {L.cdcx_kernel_name(i).decode(): (ms[i], ln[i]) for i in range(k)}

    def chain_tiers(self):
        """Segments entering each chain tier (16-lane, 64-lane, lane kernel) in the last encode."""
        out = np.zeros(3, dtype=np.int64)
        self._check(lib().cdcx_chain_tiers(self._c, _ptr(out, ctypes.c_int64)), "chain_tiers")
        return [int(x) for x in out]

    def encode_totals(self) -> dict:
        """Totals of the last device encode (cdcx_encode_totals)."""
        out = np.zeros(8, dtype=np.int64)
        self._check(lib().cdcx_encode_totals(self._c, _ptr(out, ctypes.c_int64)), "encode_totals")
        return dict(zip(["records", "matched", "runs", "with_next", "sources", "pairs", "tables", "chunks"], out.tolist()))

    def decode_tiers(self):
        """Tables entering each permutation-rebuild tier in the last decode (pair segments, whole
        table in a 16-lane group, 256-slot window, sequential list), then the number of segments,
        of segment reruns and of segments that sent their table to the next tier."""
        out = np.zeros(7, dtype=np.int64)
        self._check(lib().cdcx_decode_tiers(self._c, _ptr(out, ctypes.c_int64)), "decode_tiers")
        return [int(x) for x in out]

    def chain_stats(self):
        out = np.zeros(8, np.int64)
        self._check(lib().cdcx_chain_stats(self._c, _ptr(out, ctypes.c_int64), 8), "chain_stats")
        names = ["events", "slow_events", "winner_iters", "climb_steps", "kstar_searches", "spills", "open_steps",
                 "max_leaves"]
        return dict(zip(names, out.tolist()))

    def reset_kernel_times(self):
        self._check(lib().cdcx_reset_kernel_times(self._c), "reset_kernel_times")


# -- raw device copies for tests/bench (HIP runtime through ctypes) ------------------------
_hip = None


def hip():
    global _hip
    if _hip is None:
        for name in ("libamdhip64.so", "/opt/rocm/lib/libamdhip64.so"):
            try:
                _hip = ctypes.CDLL(name)
                break
            except OSError:
                continue
        if _hip is None:
            raise ImportError("libamdhip64.so not found")
        _hip.hipMemcpy.argtypes = [_vp, _vp, ctypes.c_size_t, ctypes.c_int]
        _hip.hipMemcpy.restype = ctypes.c_int
        _hip.hipDeviceSynchronize.restype = ctypes.c_int
        _hip.hipMalloc.argtypes = [P(_vp), ctypes.c_size_t]
        _hip.hipMalloc.restype = ctypes.c_int
        _hip.hipFree.argtypes = [_vp]
        _hip.hipFree.restype = ctypes.c_int
        _hip.hipStreamCreateWithFlags.argtypes = [P(_vp), ctypes.c_uint]
        _hip.hipStreamCreateWithFlags.restype = ctypes.c_int
        _hip.hipStreamSynchronize.argtypes = [_vp]
        _hip.hipStreamSynchronize.restype = ctypes.c_int
        _hip.hipStreamDestroy.argtypes = [_vp]
        _hip.hipStreamDestroy.restype = ctypes.c_int
        _hip.hipMemcpyAsync.argtypes = [_vp, _vp, ctypes.c_size_t, ctypes.c_int, _vp]
        _hip.hipMemcpyAsync.restype = ctypes.c_int
        _hip.hipHostMalloc.argtypes = [P(_vp), ctypes.c_size_t, ctypes.c_uint]
        _hip.hipHostMalloc.restype = ctypes.c_int
        _hip.hipHostFree.argtypes = [_vp]
        _hip.hipHostFree.restype = ctypes.c_int
    return _hip


def stream_create() -> int:
    """A non-blocking HIP stream (hipStreamNonBlocking) as an integer handle."""
    s = _vp()
    rc = hip().hipStreamCreateWithFlags(ctypes.byref(s), 1)
    if rc:
        raise CdcxError(5, f"hipStreamCreateWithFlags failed ({rc})")
    return s.value


def stream_sync(stream: int) -> None:
    rc = hip().hipStreamSynchronize(stream)
    if rc:
        raise CdcxError(5, f"hipStreamSynchronize failed ({rc})")


def stream_destroy(stream: int) -> None:
    hip().hipStreamDestroy(stream)


def memcpy_async(dst: int, src: int, nbytes: int, kind: int, stream: int) -> None:
    """kind: 1 host->device, 2 device->host, 3 device->device."""
    if nbytes:
        rc = hip().hipMemcpyAsync(dst, src, nbytes, kind, stream)
        if rc:
            raise CdcxError(5, f"hipMemcpyAsync failed ({rc})")


def replay_decode_files(contexts, paths, sink=None, batch_bytes: int = 0) -> dict:
    """Streaming replay decode of many rank files (cdcx_replay_decode_files): one host
    thread and HIP stream per context.  sink(file_index, dump_bytes) receives each file's
    table dump (the bytes cdcx_decode_stream returns) in completion order; a sink that
    raises or returns a true value stops the pipeline.  -> the call's totals."""
    L = lib()
    ctxs = (_vp * len(contexts))(*[c._c for c in contexts])
    enc = [os.fsencode(p) for p in paths]
    arr = (ctypes.c_char_p * max(len(enc), 1))(*enc)
    failure = []

    def _sink(_user, i, dump, n):
        if sink is None:
            return 0
        try:
            data = ctypes.string_at(dump, 8 * n) if n else b""
            return 1 if sink(int(i), data) else 0
        except BaseException as e:  # noqa: BLE001 - re-raised below
            failure.append(e)
            return 1

    cb = _REPLAY_SINK(_sink)
    st = ReplayStats()
    rc = L.cdcx_replay_decode_files(ctxs, len(contexts), len(enc), arr, int(batch_bytes), cb, None, ctypes.byref(st))
    if failure:
        raise failure[0]
    if rc:
        msgs = [L.cdcx_last_error(c._c).decode() for c in contexts]
        raise CdcxError(rc, "replay_decode_files: " + "; ".join(m for m in msgs if m))
    return {k: getattr(st, k) for k, _ in ReplayStats._fields_}


def _table_dict(x: Table) -> dict:
    def arr(ptr, n, dt):
        return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dt).copy() if n else np.zeros(0, dt)

    return {"set_id": x.set_id, "count": x.count, "epoch_rank": arr(x.epoch_rank, x.n_epoch, np.int64),
            "epoch_clock": arr(x.epoch_clock, x.n_epoch, np.int64),
            "with_previous": arr(x.with_previous, x.n_with_previous, np.int64),
            "matched_index": arr(x.matched_index, x.n_matched_index, np.int64),
            "unmatched_id": arr(x.unmatched_id, x.n_unmatched, np.int64),
            "unmatched_count": arr(x.unmatched_count, x.n_unmatched, np.int64),
            "ids": arr(x.ids, x.n_pairs, np.int64), "delays": arr(x.delays, x.n_pairs, np.int64),
            "perm": arr(x.perm, x.count, np.int32)}


def replay_decode_tables(contexts, paths, sink=None, batch_bytes: int = 0, convert: bool = True, footer_sink=None) -> dict:
    """Streaming replay decode delivering flat tables (cdcx_replay_decode_tables).  sink(file_index,
    chunks) gets, per file, a list (chunks) of lists (tables, ascending set id) of dicts -- copies
    of the arrays, which only live during the C callback; with convert=False the sink gets
    (file_index, n_chunks, pointer to cdcx_tables) and must not keep the pointer.
    footer_sink(file_index, {"ranks", "msg_ids", "set_ids"}) gets every file's footer right
    before its tables (cdcx_replay_decode_tables_ex)."""
    L = lib()
    ctxs = (_vp * len(contexts))(*[c._c for c in contexts])
    enc = [os.fsencode(p) for p in paths]
    arr = (ctypes.c_char_p * max(len(enc), 1))(*enc)
    failure = []

    def _sink(_user, i, n_chunks, chunks):
        if sink is None:
            return 0
        try:
            if not convert:
                return 1 if sink(int(i), int(n_chunks), chunks) else 0
            out = [[_table_dict(chunks[k].tables[q]) for q in range(chunks[k].n_tables)] for k in range(n_chunks)]
            return 1 if sink(int(i), out) else 0
        except BaseException as e:  # noqa: BLE001 - re-raised below
            failure.append(e)
            return 1

    def _fsink(_user, i, fi):
        try:
            return 1 if footer_sink(int(i), _footer_dict(fi.contents)) else 0
        except BaseException as e:  # noqa: BLE001 - re-raised below
            failure.append(e)
            return 1

    cb = _REPLAY_TABLE_SINK(_sink)
    st = ReplayStats()
    if footer_sink is None:
        rc = L.cdcx_replay_decode_tables(ctxs, len(contexts), len(enc), arr, int(batch_bytes), cb, None, ctypes.byref(st))
    else:
        fcb = _REPLAY_FOOTER_SINK(_fsink)
        rc = L.cdcx_replay_decode_tables_ex(ctxs, len(contexts), len(enc), arr, int(batch_bytes), cb, fcb, None,
                                            ctypes.byref(st))
    if failure:
        raise failure[0]
    if rc:
        msgs = [L.cdcx_last_error(c._c).decode() for c in contexts]
        raise CdcxError(rc, "replay_decode_tables: " + "; ".join(m for m in msgs if m))
    return {k: getattr(st, k) for k, _ in ReplayStats._fields_}


class PinnedBuffer:
    """Page-locked host memory (hipHostMalloc), for copy-inclusive measurements."""

    def __init__(self, nbytes: int):
        p = _vp()
        rc = hip().hipHostMalloc(ctypes.byref(p), max(nbytes, 64), 0)
        if rc:
            raise CdcxError(7, f"hipHostMalloc of {nbytes} bytes failed ({rc})")
        self.ptr = p.value
        self.nbytes = nbytes

    def close(self):
        if self.ptr:
            hip().hipHostFree(self.ptr)
            self.ptr = 0

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def d2h(ptr: int, nbytes: int, dtype=np.uint8) -> np.ndarray:
    out = np.empty(nbytes, dtype=np.uint8)
    if nbytes:
        rc = hip().hipMemcpy(out.ctypes.data, ptr, nbytes, 2)  # hipMemcpyDeviceToHost
        if rc:
            raise CdcxError(5, f"hipMemcpy D2H failed ({rc})")
    return out.view(dtype)


class DeviceArray:
    """A hipMalloc'ed copy of a host array (freed on close)."""

    def __init__(self, arr: np.ndarray):
        a = np.ascontiguousarray(arr)
        self.nbytes = a.nbytes
        p = _vp()
        rc = hip().hipMalloc(ctypes.byref(p), max(self.nbytes, 64))
        if rc:
            raise CdcxError(7, f"hipMalloc failed ({rc})")
        self.ptr = p.value
        if self.nbytes:
            rc = hip().hipMemcpy(self.ptr, a.ctypes.data, self.nbytes, 1)  # HostToDevice
            if rc:
                raise CdcxError(5, f"hipMemcpy H2D failed ({rc})")

    def close(self):
        if self.ptr:
            hip().hipFree(self.ptr)
            self.ptr = 0

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
