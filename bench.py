#!/usr/bin/env python3
"""CDC encode+decode throughput on MI355X (BASELINE.json metric).

Workload (config 3 of BASELINE.json): synthetic traces of a 1024-rank job, 10M events per
rank (gen.h / DESIGN.md "Synthetic traces").  Each GPU process holds one batch of
--ranks-per-gpu rank traces resident in HBM (they are generated on the device before the
timed region; 1024 x 10M x 32 B = 328 GB does not fit one GPU at once).  One step = CDC
encode of every rank of the batch (device bytes identical to the reference CPU encoder)
+ CDC decode of the produced files back to tables and per-table event records.
GPU g processes ranks [g*B, (g+1)*B) of the job: per-GPU work is fixed (weak scaling);
the only collective is the final reduction of counters (RCCL all-reduce over xGMI).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

Prints one JSON line (rank 0).  value = 32 B x records encoded+decoded by all GPUs /
max-over-ranks wall time of the K timed steps.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

RECORD_BYTES = 32
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--world", type=int, default=1024, help="ranks in the traced job")
    ap.add_argument("--events", type=int, default=10_000_000, help="events per rank trace")
    ap.add_argument("--ranks-per-gpu", type=int, default=96, help="rank traces resident per GPU (one step)")
    ap.add_argument("--jitter", type=int, default=8)
    ap.add_argument("--max-len", type=int, default=131072, help="REMPI_MAX")
    ap.add_argument("--verify-ranks", type=int, default=1, help="ranks checked byte-exact vs the CPU oracle")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the reference CPU CDC on a sample")
    ap.add_argument("--cpu-sample-events", type=int, default=1_000_000)
    ap.add_argument("--cpu-workers", type=int, default=16)
    ap.add_argument("--kernel-report", action="store_true", help="print per-kernel times to stderr")
    ap.add_argument("--streams", type=int, default=4, help="rank batches in flight per GPU (one HIP stream each)")
    ap.add_argument("--host-io", type=int, default=1, help="steps of the copy-inclusive measurement (0 = skip)")
    return ap.parse_args()


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


# ---------------------------------------------------------------------------------------
def cpu_baseline(args):
    """Reference CPU CDC (oracle/_ref/ref_cdc, compiled from the unmodified reference
    sources) on a bounded sample of the same workload, one process per worker core."""
    import rempi_amd

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O

    workers = max(1, min(args.cpu_workers, os.cpu_count() or 1))
    p = rempi_amd.default_gen_params(world_size=args.world, jitter=args.jitter, events_per_rank=args.cpu_sample_events)
    kind = "reference" if O.have_ref() else "port"
    tmp = tempfile.mkdtemp(prefix="cdcx_cpu_")
    recs_n = 0
    files = []
    for i in range(workers):
        r = rempi_amd.generate_host(p, i)
        recs_n += r.shape[0]
        f = os.path.join(tmp, f"rank_{i}.rec")
        r.tofile(f)
        files.append(f)
    t0 = time.perf_counter()
    if kind == "reference":
        procs = [subprocess.Popen([O.REF_BIN, "encode", f, f + ".rempi", str(args.max_len)], stdout=subprocess.PIPE,
                                  stderr=subprocess.DEVNULL) for f in files]
        enc_s = [float(pr.communicate()[0].split()[1]) for pr in procs]
        procs = [subprocess.Popen([O.REF_BIN, "decode", f + ".rempi", f + ".tables"], stdout=subprocess.PIPE,
                                  stderr=subprocess.DEVNULL) for f in files]
        dec_s = [float(pr.communicate()[0].split()[1]) for pr in procs]
    else:
        import multiprocessing as mp

        with mp.Pool(workers) as pool:
            res = pool.map(_port_one, [(f, args.max_len) for f in files])
        enc_s = [a for a, _ in res]
        dec_s = [b for _, b in res]
    wall = time.perf_counter() - t0
    for f in files:
        for ext in ("", ".rempi", ".tables"):
            try:
                os.remove(f + ext)
            except OSError:
                pass
    # Throughput on the codec's own clock (encode + decode per worker, workers in parallel)
    per_worker = [e + d for e, d in zip(enc_s, dec_s)]
    gbs = recs_n * RECORD_BYTES / max(per_worker) / 1e9
    return {"value": round(gbs, 4), "unit": "GB/s", "cores": workers, "kind": kind,
            "sample": f"{workers} rank traces x {args.cpu_sample_events} events of the same workload "
                      f"(world {args.world}, J={args.jitter}), one process per core; encode "
                      f"{np.mean(enc_s):.2f}s + decode {np.mean(dec_s):.2f}s per rank; wall {wall:.1f}s"}


def _port_one(a):
    f, mx = a
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O

    r = np.fromfile(f, dtype=np.int32).reshape(-1, 8)
    t0 = time.perf_counter()
    b, _ = O.encode(r, mx)
    t1 = time.perf_counter()
    O.decode(b)
    return t1 - t0, time.perf_counter() - t1


# ---------------------------------------------------------------------------------------
class Lane:
    """One rank batch on its own HIP stream and context (the bench runs --streams of them
    side by side, one host thread each, so one batch's latency-bound phases overlap the
    other's bandwidth-bound ones)."""

    def __init__(self, args, p, first, n, device):
        import rempi_amd
        from rempi_amd import cdcx

        self.cdcx = cdcx
        self.first, self.n = first, n
        self.stream = cdcx.stream_create()
        self.ctx = rempi_amd.Context(max_event_length=args.max_len, device=device)
        self.d_rec, self.rec_off = self.ctx.generate_device(p, first, n, stream=self.stream)
        cdcx.stream_sync(self.stream)
        self.records = int(self.rec_off[-1])
        self.comp = 0
        self.n_out = 0

    def step(self):
        c = self.ctx
        d_out, off, ln = c.encode_batch_device(self.d_rec, self.rec_off, stream=self.stream)
        d_keys, n_keys = c.batch_sorted_keys()
        _, n_out, _ = c.decode_batch_device(d_out, off, ln, d_keys, n_keys, stream=self.stream)
        self.comp += int(ln.sum())
        self.n_out = n_out
        return d_out, off, ln

    def host_io_step(self, pin_rec, pin_files, pin_recs):
        """Copy-inclusive: records H2D from pinned host memory, encode + decode, rank files
        and decoded records D2H into pinned host memory."""
        cd, c, s = self.cdcx, self.ctx, self.stream
        cd.memcpy_async(self.d_rec, pin_rec.ptr, self.records * RECORD_BYTES, 1, s)
        d_out, off, ln = c.encode_batch_device(self.d_rec, self.rec_off, stream=s)
        cd.memcpy_async(pin_files.ptr, d_out, int(off[-1] + ln[-1]), 2, s)
        d_keys, n_keys = c.batch_sorted_keys()
        d_recs, n_out, _ = c.decode_batch_device(d_out, off, ln, d_keys, n_keys, stream=s)
        cd.memcpy_async(pin_recs.ptr, d_recs, n_out * RECORD_BYTES, 2, s)
        cd.stream_sync(s)


def run_lanes(lanes, fn, steps):
    import threading

    errs = []

    def body(ln):
        try:
            for _ in range(steps):
                fn(ln)
            ln.cdcx.stream_sync(ln.stream)
        except Exception as e:  # noqa: BLE001 - re-raised on the main thread
            errs.append(e)

    ts = [threading.Thread(target=body, args=(ln,)) for ln in lanes]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errs:
        raise errs[0]


def main():
    args = parse()
    ws, rank, local = dist_env()
    import torch

    torch.cuda.set_device(local)
    dist = None
    if ws > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import rempi_amd
    from rempi_amd import cdcx

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O

    from rempi_amd import shard

    first, B = shard.shard(args.world, ws, rank, args.ranks_per_gpu)
    p = rempi_amd.default_gen_params(world_size=args.world, jitter=args.jitter, events_per_rank=args.events)
    sizes = shard.lane_sizes(B, args.streams)
    S = len(sizes)
    lanes, f = [], first
    for n in sizes:
        lanes.append(Lane(args, p, f, n, local))
        f += n
    n_records = sum(ln.records for ln in lanes)

    run_lanes(lanes, Lane.step, args.warmup)
    for ln in lanes:
        ln.comp = 0
        ln.ctx.set_profiling(True)
        ln.ctx.reset_kernel_times()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    run_lanes(lanes, Lane.step, args.steps)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    free_b, total_b = torch.cuda.mem_get_info()
    ktimes = {}
    for ln in lanes:
        ln.ctx.set_profiling(False)
        for k, (ms, nl) in ln.ctx.kernel_times().items():
            a0, b0 = ktimes.get(k, (0.0, 0))
            ktimes[k] = (a0 + ms, b0 + nl)
    comp_bytes = sum(ln.comp for ln in lanes)

    # Verification outside the timed region: byte-exact vs the CPU oracle for a sample of
    # ranks; decoded record count bounded by the input.
    fails = 0
    checked = 0
    for ln in lanes:
        d_out, off, ln_ = ln.step()
        for r in range(ln.n):
            if checked >= args.verify_ranks:
                break
            host = rempi_amd.generate_host(p, ln.first + r)
            want, _ = O.encode(host, args.max_len)
            got = cdcx.d2h(d_out + int(off[r]), int(ln_[r])).tobytes()
            fails += int(got != want)
            checked += 1
        fails += int(ln.n_out > ln.records)

    # Copy-inclusive rate (host memory in and out); never `value`.
    host_io = None
    if args.host_io and rank == 0:
        pins = []
        for ln in lanes:
            pr = cdcx.PinnedBuffer(ln.records * RECORD_BYTES)
            cdcx.memcpy_async(pr.ptr, ln.d_rec, ln.records * RECORD_BYTES, 2, ln.stream)
            cdcx.stream_sync(ln.stream)
            pins.append((pr, cdcx.PinnedBuffer(ln.records * 24 + (1 << 20)), cdcx.PinnedBuffer(ln.records * RECORD_BYTES)))
        run_lanes(lanes, lambda ln: ln.host_io_step(*pins[lanes.index(ln)]), 1)
        t1 = time.perf_counter()
        run_lanes(lanes, lambda ln: ln.host_io_step(*pins[lanes.index(ln)]), args.host_io)
        hio = time.perf_counter() - t1
        host_io = {"value": round(n_records * RECORD_BYTES * args.host_io / hio / 1e9, 3), "unit": "GB/s",
                   "steps": args.host_io,
                   "what": "H2D records from pinned host memory + encode + decode + D2H rank files and decoded records"}
        for pr in pins:
            for b in pr:
                b.close()

    counters, tmax = shard.reduce_counters([n_records * args.steps, comp_bytes, fails], elapsed, dist, "cuda")

    total_records = counters[0]
    value = total_records * RECORD_BYTES / tmax / 1e9
    comp_per_event = counters[1] / total_records

    # Roofline of the dominant kernel: algorithmic bytes per launch / mean launch time.
    kern = {k: v for k, v in ktimes.items() if v[1] > 0}
    dom = max(kern, key=lambda k: kern[k][0])
    dom_ms, dom_launches = kern[dom]
    per_launch_records = n_records / S
    algo = algorithmic_bytes(dom, per_launch_records, comp_per_event)
    achieved = algo / (dom_ms / dom_launches / 1e3) / 1e9 if dom_launches else 0.0

    if args.kernel_report and rank == 0:
        tot = sum(v[0] for v in kern.values())
        for k, (ms, n) in sorted(kern.items(), key=lambda kv: -kv[1][0]):
            print(f"  {k:22s} {ms / max(n, 1):10.3f} ms/launch x{n:4d}  {100 * ms / tot:5.1f}%", file=sys.stderr)
        print(f"  timed {elapsed:.3f}s for {args.steps} steps on {S} streams; kernels sum {tot / 1e3:.3f}s",
              file=sys.stderr)

    cpu = None
    if args.cpu_baseline and rank == 0 and ws == 1:
        cpu = cpu_baseline(args)

    if rank == 0:
        out = {
            "metric": "CDC encode+decode GB/s device-resident, 1024 ranks x 10M events; bit-exact",
            "value": round(value, 3),
            "unit": "GB/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(tmax / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic",
            "config": {"workload": f"config3: {args.world}-rank job, {args.events} events/rank traces, "
                                   f"{B} rank traces resident per GPU per step, encode+decode round trip",
                       "ranks_per_gpu": B, "events_per_rank": args.events, "records_per_step_per_gpu": n_records,
                       "jitter": args.jitter, "rempi_max": args.max_len, "streams_per_gpu": S,
                       "compressed_bytes_per_event": round(comp_per_event, 3),
                       "hbm_used_gb": round((total_b - free_b) / 1e9, 1), "hbm_total_gb": round(total_b / 1e9, 1),
                       "parallelism": f"dp{ws} (independent rank traces per GPU)",
                       "verify_failures": int(counters[2])},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": pmc_traffic(dom, per_launch_records), "traffic_source": PMC_TRAFFIC,
                         "launch_ms": round(dom_ms / dom_launches, 3),
                         "algorithmic_bytes_per_launch": round(algo),
                         "pipeline_achieved": round(pipeline_bytes(comp_per_event) * total_records / tmax / 1e9, 2)},
            "cpu_baseline": cpu,
            "host_io": host_io,
        }
        print(json.dumps(out))
    for ln in lanes:
        ln.ctx.close()
        cdcx.stream_destroy(ln.stream)
    if dist:
        dist.destroy_process_group()


# Algorithmic HBM bytes per input record for each kernel (DESIGN.md §3 kernel tables); m =
# matched fraction, c = compressed bytes per record.  The dominant kernel's figure is the
# roofline numerator.
M_FRAC = 0.833  # gen.h: one unmatched poll before 20 % of the calls -> 1 / 1.2 matched


def algorithmic_bytes(kernel, n_records, c):
    m = M_FRAC
    per = {
        "k_tile_hist": 32,
        "k_scatter": 32 + 16 + 4,
        "k_unit_prep": 16 + m * (8 + 4),
        "k_window_rank": m * (8 + 4 + 4 + 8),
        "k_sort_tiles": m * (8 + 8 + 4),
        "k_rank_tiles": m * (8 + 4 + 8 + 4 + 4 + 8),
        "k_epoch": m * 8,
        "k_chain_grp16": m * (4 + 4 + 4),
        "k_chain_grp64": m * (4 + 4 + 4),
        "k_chain_mark": m * (4 + 1),
        "k_positions": m * (4 + 1 + 4 + 4 + 4) / 2,
        "k_deltas": m * (1.3 * 4 + 0.64 * (4 + 4 + 4)),
        "k_write_units": m * (4 + 4 + 8) + c,
        "k_write_keys": m * (8 + 8),
        "k_dec_sections": 0.3 * c,
        "k_dec_perm_grp": m * (0.64 * (8 + 16) + 8),
        "k_dec_records": c + m * (4 + 8 + 8 + 1) + 32,
    }.get(kernel, 32)
    return per * n_records


PMC_TRAFFIC = "profiles/r01/pmc_traffic.json"


def pmc_traffic(kernel, n_records):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 FETCH_SIZE / WRITE_SIZE passes
    (tools/pmc_traffic.py: read bytes = 2 x FETCH_SIZE per the gfx950 correction, checked on
    k_tile_hist), scaled to the records one launch processes; None if not collected."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), PMC_TRAFFIC)
    try:
        k = json.load(open(path))["kernels"].get(kernel)
    except (OSError, ValueError, KeyError):
        return None
    return None if k is None else round(k["bytes_per_record"] * n_records)


def pipeline_bytes(c):
    """encode reads 32 B/event and writes c; decode reads c + 8m of sorted keys
    and writes 32 B/event."""
    return 64 + 2 * c + 8 * M_FRAC


if __name__ == "__main__":
    main()
