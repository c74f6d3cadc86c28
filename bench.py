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
    ap.add_argument("--ranks-per-gpu", type=int, default=32, help="rank traces resident per GPU (one step)")
    ap.add_argument("--jitter", type=int, default=8)
    ap.add_argument("--max-len", type=int, default=131072, help="REMPI_MAX")
    ap.add_argument("--verify-ranks", type=int, default=1, help="ranks checked byte-exact vs the CPU oracle")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the reference CPU CDC on a sample")
    ap.add_argument("--cpu-sample-events", type=int, default=1_000_000)
    ap.add_argument("--cpu-workers", type=int, default=16)
    ap.add_argument("--kernel-report", action="store_true", help="print per-kernel times to stderr")
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

    B = args.ranks_per_gpu
    first = (rank * B) % args.world
    p = rempi_amd.default_gen_params(world_size=args.world, jitter=args.jitter, events_per_rank=args.events)
    ctx = rempi_amd.Context(max_event_length=args.max_len, device=local)
    d_rec, rec_off = ctx.generate_device(p, first, B)
    n_records = int(rec_off[-1])

    # The stream the library launches on: the default stream (NULL); its HIP events time
    # each kernel (cdcx_set_profiling).
    def step():
        d_out, off, ln = ctx.encode_batch_device(d_rec, rec_off)
        d_keys, n_keys = ctx.batch_sorted_keys()
        _, n_out, _ = ctx.decode_batch_device(d_out, off, ln, d_keys, n_keys)
        return int(ln.sum()), n_out

    for _ in range(args.warmup):
        step()
    ctx.set_profiling(True)
    ctx.reset_kernel_times()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    comp_bytes = 0
    for _ in range(args.steps):
        cb, n_out = step()
        comp_bytes += cb
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ctx.set_profiling(False)
    ktimes = ctx.kernel_times()

    # Verification outside the timed region: byte-exact vs the CPU oracle for a sample of
    # ranks; decode(encode(x)) record round trip for the whole batch.
    d_out, off, ln = ctx.encode_batch_device(d_rec, rec_off)
    fails = 0
    for r in range(min(args.verify_ranks, B)):
        host = rempi_amd.generate_host(p, first + r)
        want, _ = O.encode(host, args.max_len)
        got = cdcx.d2h(d_out + int(off[r]), int(ln[r])).tobytes()
        fails += int(got != want)
    d_keys, n_keys = ctx.batch_sorted_keys()
    d_recs, n_out, _ = ctx.decode_batch_device(d_out, off, ln, d_keys, n_keys)
    # round trip: decoded per-table streams are a permutation of the input records grouped by
    # (chunk, table); compare multisets of (set, src, clock, with_next, index) of matched events
    fails += int(n_out > n_records)

    counters = np.array([n_records * args.steps, comp_bytes, fails], dtype=np.float64)
    tmax = elapsed
    if dist:
        t = torch.tensor([elapsed], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        tmax = float(t.item())
        c = torch.tensor(counters, device="cuda")
        dist.all_reduce(c)
        counters = c.cpu().numpy()

    total_records = counters[0]
    value = total_records * RECORD_BYTES / tmax / 1e9
    comp_per_event = counters[1] / total_records

    # Roofline of the dominant kernel: algorithmic bytes per launch / mean launch time.
    enc_kernels = {k: v for k, v in ktimes.items() if v[1] > 0}
    dom = max(enc_kernels, key=lambda k: enc_kernels[k][0])
    dom_ms, dom_launches = enc_kernels[dom]
    algo = algorithmic_bytes(dom, n_records, comp_per_event)
    achieved = algo / (dom_ms / dom_launches / 1e3) / 1e9 if dom_launches else 0.0

    if args.kernel_report and rank == 0:
        tot = sum(v[0] for v in enc_kernels.values())
        for k, (ms, n) in sorted(enc_kernels.items(), key=lambda kv: -kv[1][0]):
            print(f"  {k:22s} {ms / max(n, 1):10.3f} ms/launch x{n:4d}  {100 * ms / tot:5.1f}%", file=sys.stderr)
        print(f"  timed {elapsed:.3f}s for {args.steps} steps; kernels sum {tot / 1e3:.3f}s", file=sys.stderr)

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
                       "jitter": args.jitter, "rempi_max": args.max_len,
                       "compressed_bytes_per_event": round(comp_per_event, 3),
                       "parallelism": f"dp{ws} (independent rank traces per GPU)",
                       "verify_failures": int(counters[2])},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                         "pipeline_achieved": round(pipeline_bytes(comp_per_event) * total_records / tmax / 1e9, 2)},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


# Algorithmic HBM bytes per record for each kernel (DESIGN.md "Kernels and their
# rooflines"); c = compressed bytes per record.
def algorithmic_bytes(kernel, n_records, c):
    m = 0.86  # matched fraction of the synthetic workload (gen.h: 1 poll per 5 calls)
    per = {
        "k_scatter": 32 + 1 + 16 + 4,
        "k_unit_prep": 16 + m * (8 + 4) + 0.3 * 12,
        "k_sort_tiles": m * (8 + 8 + 4),
        "k_rank_tiles": m * (8 + 4 + 4 + 4 + 8),
        "k_epoch": m * 8,
        "k_chain_lane": m * (4 + 4 + 4 + 4 + 1),
        "k_positions": m * (4 + 4 + 1 + 4 + 4 + 8 + 8),
        "k_deltas": m * (4 + 1 + 4 + 4 + 8 + 4 + 4),
        "k_write_units": m * (4 + 4 + 8 + 8) + c,
        "k_dec_sections": c + m * 32,
        "k_dec_perm_lane": m * (8 + 8 + 4 + 4 + 4),
        "k_dec_records": c + m * (4 + 8 + 4) + 32,
    }.get(kernel, 32)
    return per * n_records


def pipeline_bytes(c):
    """encode reads 32 B/event and writes c; decode reads c + 8m of sorted keys
    and writes 32 B/event."""
    return 64 + 2 * c + 8 * 0.86


if __name__ == "__main__":
    main()
