"""Diagnostics: run one encode of a synthetic batch with chain-kernel counters enabled."""
import os, sys
os.environ["CDCX_CHAIN_STATS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import rempi_amd
from rempi_amd import cdcx
ranks = int(sys.argv[1]) if len(sys.argv) > 1 else 8
jit = int(sys.argv[2]) if len(sys.argv) > 2 else 8
p = rempi_amd.default_gen_params(world_size=1024, jitter=jit, events_per_rank=10_000_000)
c = rempi_amd.Context()
d, off = c.generate_device(p, 0, ranks)
import ctypes
L = cdcx.lib()
# zero the stats buffer through a first encode, then read after a second one
c.encode_batch_device(d, off)
c.chain_stats()
c.set_profiling(True); c.reset_kernel_times()
c.encode_batch_device(d, off)
kt = c.kernel_times()
print("k_chain_seg ms", kt["k_chain_seg"], "ranks", ranks, "jitter", jit)
print(c.chain_stats())
