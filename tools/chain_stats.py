"""Path counts of the 8-lane chain kernel on a bench-shaped batch (profiling build only):
build rempi_amd/libcdcx_stats.so with -DCDCX_CHAIN_STATS, then
CDCX_LIB=libcdcx_stats.so python tools/chain_stats.py [ranks]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import rempi_amd  # noqa: E402
from rempi_amd import cdcx  # noqa: E402

NAMES = ["wave iterations", "fetch path", "body", "useB", "binsearch", "binsearch steps", "ks>=1", "need", "climb steps A",
         "interior ok", "root", "exta", "topg spill (grow)", "topg update", "qn store", "sweep path", "sweep compaction A",
         "sweep compaction B", "overflow", "ring reads > 16 rows back", "segments fetched", "active lanes in body", "ring reads > 64 rows back (global)", "ring reads > 32 rows back"]

ranks = int(sys.argv[1]) if len(sys.argv) > 1 else 8
p = rempi_amd.default_gen_params(world_size=1024, events_per_rank=10_000_000)
ctx = rempi_amd.Context(max_event_length=131072, device=0)
s = cdcx.stream_create()
d_rec, rec_off = ctx.generate_device(p, 0, ranks, stream=s)
cdcx.stream_sync(s)
L = cdcx.lib()
L.cdcx_debug_g8_stats.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
out = (ctypes.c_ulonglong * 24)()
L.cdcx_debug_g8_stats(out, 1)
ctx.encode_batch_device(d_rec, rec_off, stream=s)
cdcx.stream_sync(s)
L.cdcx_debug_g8_stats(out, 1)
it = max(out[2], 1)
for k, n in enumerate(NAMES):
    if n:
        print(f"{n:24s} {out[k]:14d}  {out[k] / it:8.4f} per body iteration")
