#!/usr/bin/env python3
"""CDC encode+decode throughput on MI355X (BASELINE.json metric).

Workload (configs 3/4 of BASELINE.json): synthetic traces of a 1024-rank job, 10M events per
rank (rempi_amd/csrc/gen.h): 327.7 GB of records, more than one GPU's HBM.
The job's ranks are sharded over the GPUs in contiguous blocks (rank r -> GPU floor(r G / R),
rempi_amd/shard.py); each GPU process walks its block in batches of at most --ranks-per-gpu
rank traces resident in HBM.  Per batch: the traces are generated on the device (untimed),
then W warmup and K timed steps run with inputs and outputs resident.  One step of a batch =
CDC encode of every rank of the batch (device bytes identical to the reference CPU encoder)
+ CDC decode of the produced files back to tables and per-table event records; one step of
the job = one step of every batch.  The timed regions of the batches are summed.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

Prints one JSON line (rank 0).  value = 32 B x records encoded+decoded by all GPUs in the K
steps / max-over-ranks timed seconds.  The total work is the whole job whatever N is
("strong" scaling); the only collective is the final reduction of counters (RCCL all-reduce).

After the timed steps of a batch every rank is verified (outside the timed region): the
decoded records of all ranks are compared on the device with the input they must reproduce,
and the ranks pinned by tests/golden/config3_full.json (hashes of the reference encoder's
file, the reference decoder's permutation and the expected records at full size) are hashed.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

RECORD_BYTES = 32
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
SIMDS = 1024           # 256 CUs x 4 SIMDs
SCLK_HZ = 2.4e9        # engine clock under this load (rocm-smi during the bench: 2.35-2.40 GHz)
FIXTURE = os.path.join(ROOT, "tests", "golden", "config3_full.json")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--world", type=int, default=1024, help="ranks in the traced job")
    ap.add_argument("--events", type=int, default=10_000_000, help="events per rank trace")
    ap.add_argument("--ranks-per-gpu", type=int, default=128, help="rank traces resident per GPU (one batch)")
    ap.add_argument("--jitter", type=int, default=8)
    ap.add_argument("--max-len", type=int, default=131072, help="REMPI_MAX")
    ap.add_argument("--streams", type=int, default=8, help="lanes of a batch in flight per GPU (one HIP stream each)")
    ap.add_argument("--max-batches", type=int, default=0,
                    help="process only the first B batches of each GPU's block (0 = the whole block)")
    ap.add_argument("--verify", type=int, default=1, help="verify every rank after the timed steps of its batch")
    ap.add_argument("--oracle-ranks", type=int, default=1, help="ranks also encoded by the CPU oracle and compared")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the reference CPU CDC on a sample")
    ap.add_argument("--cpu-sample-ranks", type=int, default=64, help="rank traces of the CPU sample (config 2: 64)")
    ap.add_argument("--cpu-sample-events", type=int, default=1_000_000, help="events per rank of the CPU sample")
    ap.add_argument("--cpu-workers", type=int, default=0, help="CPU worker processes (0 = the cores this process may use)")
    ap.add_argument("--kernel-report", action="store_true", help="print per-kernel times to stderr")
    ap.add_argument("--host-io", type=int, default=1, help="steps of the copy-inclusive measurement (0 = skip)")
    ap.add_argument("--host-io-ranks", type=int, default=12, help="rank traces per lane (of at most four) in the copy-inclusive measurement")
    ap.add_argument("--config2", type=int, default=-1,
                    help="also run config 2 (the CPU sample's 64 x 1M traces) on the GPU and compare its files with the CPU "
                         "codec's (default: when the CPU baseline runs)")
    ap.add_argument("--solo", type=int, default=2, help="steps of one lane alone for the roofline figure (0 = skip)")
    ap.add_argument("--solo-ranks", type=int, default=32,
                    help="rank traces of that launch: enough to keep the GPU full for the whole kernel (a lane of the timed "
                         "steps holds ranks-per-gpu / streams, whose chain kernel alone ends in the tail of its longest segments)")
    return ap.parse_args(argv)


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


# ---------------------------------------------------------------------------------------
def usable_cores() -> int:
    """CPUs this process may run on (the GPU box grants a share of the host, which
    os.cpu_count() does not show; OMP_NUM_THREADS carries it there)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    for var in ("OMP_NUM_THREADS", "MAX_JOBS"):
        v = os.environ.get(var, "")
        if v.isdigit() and int(v) > 0:
            n = min(n, int(v))
    return max(1, n)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(args):
    """Reference CPU CDC (oracle/_ref/ref_cdc, compiled from the unmodified reference sources;
    the C++ restatement when that binary is absent) on config 2 of BASELINE.json -- 64 rank
    traces x 1M events of the same generator -- one worker process per usable core, encode and
    decode timed separately on the codec's own clock (trace loading and event construction
    excluded, as the GPU figure excludes generation)."""
    import rempi_amd

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O

    workers = args.cpu_workers or usable_cores()
    n = args.cpu_sample_ranks
    p = rempi_amd.default_gen_params(world_size=args.world, jitter=args.jitter, events_per_rank=args.cpu_sample_events)
    kind = "reference" if O.have_ref() else "port"
    tmp = tempfile.mkdtemp(prefix="cdcx_cpu_")
    files, recs_n = [], 0
    for i in range(n):
        r = rempi_amd.generate_host(p, i)
        recs_n += r.shape[0]
        f = os.path.join(tmp, f"rank_{i}.rec")
        r.tofile(f)
        files.append(f)
    enc_s, dec_s = [0.0] * n, [0.0] * n
    busy = [0.0] * workers  # codec seconds per worker
    nxt = [0]
    lock = threading.Lock()

    file_sha = [None] * n  # SHA-256 of every rank file the CPU codec wrote (config2's byte comparison)

    def one(f):
        if kind == "reference":
            a = subprocess.run([O.REF_BIN, "encode", f, f + ".rempi", str(args.max_len)], capture_output=True, text=True)
            b = subprocess.run([O.REF_BIN, "decode", f + ".rempi", f + ".tables"], capture_output=True, text=True)
            with open(f + ".rempi", "rb") as fh:
                file_sha[files.index(f)] = hashlib.sha256(fh.read()).hexdigest()
            return float(a.stdout.split()[1]), float(b.stdout.split()[1])
        out = subprocess.run([sys.executable, os.path.abspath(__file__), "--port-one", f, str(args.max_len)],
                             capture_output=True, text=True)
        e, d, sha = out.stdout.split()[-3:]
        file_sha[files.index(f)] = sha
        return float(e), float(d)

    def work(w):
        while True:
            with lock:
                i = nxt[0]
                nxt[0] += 1
            if i >= n:
                return
            enc_s[i], dec_s[i] = one(files[i])
            busy[w] += enc_s[i] + dec_s[i]

    t0 = time.perf_counter()
    ts = [threading.Thread(target=work, args=(w,)) for w in range(workers)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    wall = time.perf_counter() - t0
    for f in files:
        for ext in ("", ".rempi", ".tables"):
            try:
                os.remove(f + ext)
            except OSError:
                pass
    try:
        os.rmdir(tmp)
    except OSError:
        pass
    nbytes = recs_n * RECORD_BYTES
    return {"value": round(nbytes / max(busy) / 1e9, 4), "unit": "GB/s", "cores": workers, "kind": kind,
            "encode_gbs": round(nbytes / (sum(enc_s) / workers) / 1e9, 4),
            "decode_gbs": round(nbytes / (sum(dec_s) / workers) / 1e9, 4),
            "encode_s_per_rank": round(float(np.mean(enc_s)), 3), "decode_s_per_rank": round(float(np.mean(dec_s)), 3),
            "wall_s": round(wall, 2), "wall_gbs": round(nbytes / wall / 1e9, 4),
            "cpu_model": cpu_model(), "host_cpus": os.cpu_count(), "usable_cpus": usable_cores(),
            "file_sha256": file_sha,
            "sample": f"config 2 in full: {n} rank traces x {args.cpu_sample_events} events of the same workload "
                      f"(world {args.world}, J={args.jitter}), {workers} worker processes; value = bytes / "
                      f"(encode + decode codec seconds of the busiest worker)"}


def port_one(f, mx):
    """Child of cpu_baseline when the reference binary is absent: the C++ restatement."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O

    r = np.fromfile(f, dtype=np.int32).reshape(-1, 8)
    t0 = time.perf_counter()
    b, _ = O.encode(r, mx)
    t1 = time.perf_counter()
    O.decode(b)
    print(t1 - t0, time.perf_counter() - t1, hashlib.sha256(b).hexdigest())


# ---------------------------------------------------------------------------------------
class Lane:
    """One lane of a batch: a rank sub-batch on its own HIP stream and context (a batch runs
    --streams of them side by side, one host thread each, so one lane's latency-bound phases
    overlap another's bandwidth-bound ones)."""

    def __init__(self, max_len, device):
        import rempi_amd
        from rempi_amd import cdcx

        self.cdcx = cdcx
        self.stream = cdcx.stream_create()
        self.ctx = rempi_amd.Context(max_event_length=max_len, device=device)
        self.first = self.n = self.records = 0
        self.comp = 0
        self.last = None

    def load(self, p, first, n):
        """Generate ranks [first, first + n) of the job into this lane's device buffer."""
        self.first, self.n = first, n
        self.d_rec, self.rec_off = self.ctx.generate_device(p, first, n, stream=self.stream)
        self.cdcx.stream_sync(self.stream)
        self.records = int(self.rec_off[-1])

    def step(self):
        c = self.ctx
        d_out, off, ln = c.encode_batch_device(self.d_rec, self.rec_off, stream=self.stream)
        d_keys, n_keys = c.batch_sorted_keys()
        d_recs, n_out, d_perm = c.decode_batch_device(d_out, off, ln, d_keys, n_keys, stream=self.stream)
        self.comp += int(ln.sum())
        self.last = (d_out, off, ln, d_recs, n_out, d_perm)

    def totals(self):
        return self.ctx.encode_totals()

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

    def close(self):
        self.ctx.close()
        self.cdcx.stream_destroy(self.stream)


STAGGER_S = float(os.environ.get("CDCX_BENCH_STAGGER_MS", "0")) / 1e3  # experiment: lane k starts k * this later
PROFILE_TIMED = os.environ.get("CDCX_BENCH_NOPROF", "0") == "0"  # experiment: HIP events around every kernel of the timed steps


def run_lanes(lanes, fn, steps):
    errs = []

    def body(ln):
        try:
            if STAGGER_S:
                time.sleep(STAGGER_S * lanes.index(ln))
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


# ---------------------------------------------------------------------------------------
def load_fixture(args):
    """Reference hashes of full-size ranks, if they describe this run's workload."""
    try:
        fx = json.load(open(FIXTURE))
    except (OSError, ValueError):
        return {}
    g = fx["generator"]
    if (g["world_size"], g["events_per_rank"], g["jitter"], fx["max_len"]) != (args.world, args.events, args.jitter,
                                                                               args.max_len):
        return {}
    return {int(k): v for k, v in fx["ranks"].items()}


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(memoryview(np.ascontiguousarray(a))).hexdigest()


def verify_lane(ln: Lane, fixture: dict, oracle_ranks=(), p=None, max_len=131072) -> dict:
    """Checks of the lane's last step (outside any timed region).
    decode: every rank's decoded records against the input on the device (round trip), the
            decoded record count, and -- for ranks the fixture pins -- SHA-256 of the records
            and of the permutation against the reference decoder's.
    encode: for fixture ranks, SHA-256 and length of the rank file against the reference
            encoder's; for `oracle_ranks`, the bytes against the CPU restatement."""
    cd = ln.cdcx
    d_out, off, flen, d_recs, n_out, d_perm = ln.last
    res = {"enc_ranks": 0, "enc_fail": 0, "dec_ranks": ln.n, "dec_fail": 0, "notes": []}
    bad = ln.ctx.verify_roundtrip_device(ln.d_rec, stream=ln.stream)
    if bad or n_out != ln.records:
        res["dec_fail"] += ln.n
        res["notes"].append(f"lane at rank {ln.first}: {bad} decoded records differ, {n_out} of {ln.records} records")
    ro, po = ln.ctx.decode_rank_offsets(ln.n)
    for q in range(ln.n):
        r = ln.first + q
        fx = fixture.get(r)
        if fx is not None:
            res["enc_ranks"] += 1
            data = cd.d2h(d_out + int(off[q]), int(flen[q]))
            if int(flen[q]) != fx["file_len"] or sha(data) != fx["file_sha256"]:
                res["enc_fail"] += 1
                res["notes"].append(f"rank {r}: file differs from the reference encoder's")
            recs = cd.d2h(d_recs + int(ro[q]) * RECORD_BYTES, int(ro[q + 1] - ro[q]) * RECORD_BYTES)
            perm = cd.d2h(d_perm + int(po[q]) * 4, int(po[q + 1] - po[q]) * 4)
            if int(ro[q + 1] - ro[q]) != fx["records_out"] or sha(recs) != fx["records_sha256"] or \
                    int(po[q + 1] - po[q]) != fx["matched"] or sha(perm) != fx["perm_sha256"]:
                res["dec_fail"] += 1
                res["notes"].append(f"rank {r}: decoded records / permutation differ from the reference's")
        if r in oracle_ranks:
            import rempi_amd

            sys.path.insert(0, os.path.join(ROOT, "tests"))
            import oracle_lib as O

            want, _ = O.encode(rempi_amd.generate_host(p, r), max_len)
            res["enc_ranks"] += 0 if fx is not None else 1
            if cd.d2h(d_out + int(off[q]), int(flen[q])).tobytes() != want:
                res["enc_fail"] += 1
                res["notes"].append(f"rank {r}: file differs from the CPU restatement's")
    return res


def run_config2(args, device, file_sha, steps=6):
    """Config 2 of BASELINE.json on the GPU, beside the CPU leg that runs it in full: the 64 rank
    traces x 1M events of the same generator, one resident batch on up to four lanes, encoded and
    decoded `steps` times (timed, device-resident), every rank verified by the device round trip,
    and every rank file compared (SHA-256) with the one the CPU codec wrote for that rank."""
    import torch

    import rempi_amd
    from rempi_amd import cdcx, shard

    n = args.cpu_sample_ranks
    p = rempi_amd.default_gen_params(world_size=args.world, jitter=args.jitter, events_per_rank=args.cpu_sample_events)
    lanes = [Lane(args.max_len, device) for _ in range(max(1, min(args.streams, 4, n)))]  # (16 traces of 1 M events per lane)
    try:
        at = 0
        for ln, k in zip(lanes, shard.lane_sizes(n, len(lanes))):
            ln.load(p, at, k)
            at += k
        run_lanes(lanes, Lane.step, 1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run_lanes(lanes, Lane.step, steps)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        records = sum(ln.records for ln in lanes)
        bad_rt = cmp_n = cmp_bad = 0
        for ln in lanes:
            d_out, off, flen, d_recs, n_out, d_perm = ln.last
            if ln.ctx.verify_roundtrip_device(ln.d_rec, stream=ln.stream) or n_out != ln.records:
                bad_rt += ln.n
            for q in range(ln.n):
                want = file_sha[ln.first + q] if file_sha else None
                if want:
                    cmp_n += 1
                    cmp_bad += sha(cdcx.d2h(d_out + int(off[q]), int(flen[q]))) != want
        return {"workload": f"config2: {n} rank traces x {args.cpu_sample_events} events (world {args.world}, J={args.jitter}), "
                            f"one resident batch on {len(lanes)} lanes, encode+decode round trip",
                "value": round(records * steps * RECORD_BYTES / dt / 1e9, 3), "unit": "GB/s", "steps": steps,
                "ms_per_step": round(dt / steps * 1e3, 3), "records_per_step": records,
                "verify": {"roundtrip_ranks": n, "roundtrip_failures": bad_rt, "files_compared_with_cpu_codec": cmp_n,
                           "file_failures": int(cmp_bad)}}
    finally:
        for ln in lanes:
            ln.close()


# ---------------------------------------------------------------------------------------
def main():
    args = parse()
    ws, rank, local = dist_env()
    # One hardware queue per lane: with HIP's default of 4 two lanes share a queue and run one behind
    # the other (5 lanes on 4 queues are slower than 4).  Read when the HIP runtime starts, so set
    # before anything touches the GPU.
    want_q = min(16, max(4, args.streams))
    have_q = os.environ.get("GPU_MAX_HW_QUEUES", "")
    if not have_q.isdigit() or int(have_q) < want_q:
        os.environ["GPU_MAX_HW_QUEUES"] = str(want_q)
    import torch

    # One process per GPU over RCCL.  CDCX_BENCH_BACKEND=gloo is the rehearsal of the N > 1 path
    # on a box with fewer GPUs than processes: the processes share the GPUs round robin and the
    # final reduction runs on host tensors.
    backend = os.environ.get("CDCX_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dist = None
    if ws > 1:
        import torch.distributed as dist

        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    import rempi_amd
    from rempi_amd import cdcx, shard

    shard.check_cover(args.world, ws)
    first, count = shard.block(args.world, ws, rank)
    plan = shard.batches(first, count, args.ranks_per_gpu)
    if args.max_batches > 0:
        plan = plan[:args.max_batches]
    p = rempi_amd.default_gen_params(world_size=args.world, jitter=args.jitter, events_per_rank=args.events)
    fixture = load_fixture(args) if args.verify else {}
    lanes = [Lane(args.max_len, local) for _ in range(max(1, min(args.streams, args.ranks_per_gpu)))]
    n_lanes = len(lanes)

    elapsed = 0.0
    n_records = comp_bytes = n_matched = n_pairs = 0
    ver = {"enc_ranks": 0, "enc_fail": 0, "dec_ranks": 0, "dec_fail": 0, "notes": []}
    ktimes = {}
    per_launch_records = 0
    oracle_left = args.oracle_ranks if (args.verify and rank == 0) else 0
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t_job = time.perf_counter()
    active = lanes
    for (b_first, b_n) in plan:
        sizes = shard.lane_sizes(b_n, len(lanes))
        active = lanes[:len(sizes)]
        at = b_first
        for ln, n in zip(active, sizes):
            ln.load(p, at, n)
            at += n
        run_lanes(active, Lane.step, args.warmup)
        for ln in active:
            ln.comp = 0
            ln.ctx.set_profiling(PROFILE_TIMED)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run_lanes(active, Lane.step, args.steps)
        torch.cuda.synchronize()
        elapsed += time.perf_counter() - t0
        for ln in active:
            ln.ctx.set_profiling(False)
            n_records += ln.records
            comp_bytes += ln.comp
            t = ln.totals()
            n_matched += t["matched"]
            n_pairs += t["pairs"]
        per_launch_records = max(per_launch_records, max(ln.records for ln in active))
        if args.verify:
            for ln in active:
                take = list(range(ln.first, ln.first + min(oracle_left, ln.n)))
                oracle_left -= len(take)
                v = verify_lane(ln, fixture, take, p, args.max_len)
                for k in ("enc_ranks", "enc_fail", "dec_ranks", "dec_fail"):
                    ver[k] += v[k]
                ver["notes"] += v["notes"]
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    job_wall = time.perf_counter() - t_job
    free_b, total_b = torch.cuda.mem_get_info()
    for ln in lanes:
        for k, (ms, nl) in ln.ctx.kernel_times().items():
            a0, b0 = ktimes.get(k, (0.0, 0))
            ktimes[k] = (a0 + ms, b0 + nl)
        ln.ctx.reset_kernel_times()

    chain_tiers0 = lanes[0].ctx.chain_tiers()  # (of the timed steps: the legs below reload the lanes)
    decode_tiers = [ln.ctx.decode_tiers() for ln in lanes]

    # Copy-inclusive rate (host memory in and out); never `value`.
    host_io = None
    if args.host_io and rank == 0 and active:
        pins = []
        active = active[:4]  # (four lanes fill the PCIe link; more only split it)
        for ln in active:  # a bounded sample: 88 B of pinned host memory per record
            if ln.n > args.host_io_ranks:
                ln.load(p, ln.first, args.host_io_ranks)
            pr = cdcx.PinnedBuffer(ln.records * RECORD_BYTES)
            cdcx.memcpy_async(pr.ptr, ln.d_rec, ln.records * RECORD_BYTES, 2, ln.stream)
            cdcx.stream_sync(ln.stream)
            pins.append((pr, cdcx.PinnedBuffer(ln.records * 24 + (1 << 20)), cdcx.PinnedBuffer(ln.records * RECORD_BYTES)))
        run_lanes(active, lambda ln: ln.host_io_step(*pins[active.index(ln)]), 1)
        t1 = time.perf_counter()
        run_lanes(active, lambda ln: ln.host_io_step(*pins[active.index(ln)]), args.host_io)
        hio = time.perf_counter() - t1
        nb = sum(ln.records for ln in active) * RECORD_BYTES * args.host_io
        host_io = {"value": round(nb / hio / 1e9, 3), "unit": "GB/s", "steps": args.host_io,
                   "ranks": sum(ln.n for ln in active),
                   "what": "H2D records from pinned host memory + encode + decode + D2H rank files and decoded records"}
        for pr in pins:
            for b in pr:
                b.close()

    # Dominant kernel alone on the GPU (one lane, nothing else in flight): its launch duration
    # for the roofline figure.  Under --streams lanes the HIP events of a launch also cover the
    # time the lane shares the CUs with the other lanes.  The other lanes are closed first, so
    # that the one lane can hold --solo-ranks traces.
    solo = {}
    if args.solo and rank == 0 and active:
        for ln in lanes[1:]:
            ln.close()
        lanes = lanes[:1]
        ln = lanes[0]
        want = max(1, min(args.solo_ranks, args.ranks_per_gpu, count))
        if ln.n != want:
            ln.load(p, first, want)
        run_lanes([ln], Lane.step, 1)
        ln.ctx.reset_kernel_times()
        ln.ctx.set_profiling(True)
        run_lanes([ln], Lane.step, args.solo)
        ln.ctx.set_profiling(False)
        solo = {k: v for k, v in ln.ctx.kernel_times().items() if v[1] > 0}
        solo_records = ln.records

    counters, tmax = shard.reduce_counters(
        [n_records * args.steps, comp_bytes, ver["enc_ranks"], ver["enc_fail"], ver["dec_ranks"], ver["dec_fail"],
         count if args.max_batches <= 0 else sum(n for _, n in plan), n_records, n_matched, n_pairs], elapsed, dist,
        "cuda" if backend == "nccl" else "cpu")
    if dist:  # the last collective is done: what follows (CPU baseline, config 2, the JSON line) is rank 0's alone
        dist.barrier()
        dist.destroy_process_group()
        dist = None
    total_records = counters[0]
    value = total_records * RECORD_BYTES / tmax / 1e9
    comp_per_event = counters[1] / max(total_records, 1)
    # matched events per record and (id, delay) pairs per matched event, from the encoders' own totals
    mix = Mix(m=counters[8] / max(counters[7], 1), pairs=counters[9] / max(counters[8], 1), c=comp_per_event)

    # Roofline of the dominant kernel: algorithmic bytes per launch / mean launch duration.
    # Dominant = the longest launch with the GPU to itself (the solo steps); with all lanes in
    # flight a launch's duration also counts the time its waves wait for the other lanes'.
    kern = {k: v for k, v in ktimes.items() if v[1] > 0}
    traffic = pmc_traffic() if rank == 0 else None

    def line(k, launch_ms, launch_records):
        algo = algorithmic_bytes(k, launch_records, mix)
        d = {"kernel": k, "launch_ms": round(launch_ms, 3), "algorithmic_bytes_per_launch": None, "achieved": None,
             "frac": None, "bound": KERNEL_BOUND.get(k, "hbm")}
        if algo is not None:  # (kernels that touch a data-dependent part of the batch have no per-record figure)
            ach = algo / (launch_ms / 1e3) / 1e9
            d.update({"algorithmic_bytes_per_launch": round(algo), "achieved": round(ach, 2),
                      "frac": round(ach / HBM_PEAK_GBS, 5)})
        pk = (traffic or {}).get("kernels", {}).get(k)
        if pk and pk.get("bytes_per_record") is not None:
            d["traffic"] = round(pk["bytes_per_record"] * launch_records)
            # vector-instruction issue: wave instructions x 4 cycles on the chip's SIMDs
            issue_s = pk["valu"] / traffic["records"] * launch_records * 4 / (SIMDS * SCLK_HZ)
            d["valu_issue_frac"] = round(issue_s / (launch_ms / 1e3), 3)
        return d

    if solo:
        per = {k: (v[0] / v[1], solo_records) for k, v in solo.items()}
    else:
        per = {k: (v[0] / v[1], per_launch_records) for k, v in kern.items()}
    order = sorted(per, key=lambda k: -per[k][0])
    if order:
        dom = order[0]
        dom_ms, dom_launches = kern.get(dom, (0.0, 0))
        launch_ms, launch_records = per[dom]
        dom_line = line(dom, launch_ms, launch_records)
        top = [line(k, *per[k]) for k in order[:8]]
    else:  # no kernel was timed (no solo steps and no per-kernel events)
        dom, dom_ms, dom_launches, launch_ms, top = None, 0.0, 0, 0.0, []
        dom_line = {"achieved": None, "frac": None, "algorithmic_bytes_per_launch": None}

    if args.kernel_report and rank == 0:
        tot = sum(v[0] for v in kern.values())
        for k, (ms, n) in sorted(kern.items(), key=lambda kv: -kv[1][0]):
            so = solo.get(k)
            print(f"  {k:22s} {ms / max(n, 1):10.3f} ms/launch x{n:5d}  {100 * ms / tot:5.1f}%"
                  + (f"   alone {so[0] / so[1]:8.3f} ms" if so else ""), file=sys.stderr)
        if solo:
            print(f"  (per launch: {per_launch_records} records with all lanes in flight, {solo_records} alone)", file=sys.stderr)
        print(f"  timed {elapsed:.3f}s for {args.steps} steps x {len(plan)} batches on {n_lanes} streams; "
              f"kernels sum {tot / 1e3:.3f}s; job wall {job_wall:.1f}s", file=sys.stderr)
        print(f"  chain tiers of the last encode of lane 0 (segments: all, past 16 leaves, past 64): "
              f"{chain_tiers0}", file=sys.stderr)
        print(f"  rebuild tiers of the lanes' last decodes (tables: all, whole-table groups, window, list; segments: all, "
              f"rerun, given up): {decode_tiers}", file=sys.stderr)
        for note in ver["notes"][:20]:
            print("  verify:", note, file=sys.stderr)

    # (after the last collective: with several GPU processes only rank 0 is still busy here)
    cpu = cfg2 = None
    if args.cpu_baseline and rank == 0:
        cpu = cpu_baseline(args)
    if (args.config2 if args.config2 >= 0 else args.cpu_baseline) and rank == 0:
        for ln in lanes:  # (their buffers hold most of the HBM)
            ln.close()
        lanes = []
        cfg2 = run_config2(args, local, (cpu or {}).get("file_sha256"))
    if cpu:
        cpu.pop("file_sha256", None)

    if rank == 0:
        ranks_done = int(counters[6])
        out = {
            "metric": "CDC encode+decode GB/s device-resident, 1024 ranks x 10M events; bit-exact",
            "value": round(value, 3),
            "unit": "GB/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(tmax / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic",
            "config": {"workload": f"config3/4: {args.world}-rank job x {args.events} events/rank, {ranks_done} rank traces "
                                   f"processed per step over {ws} GPU(s) in batches of <= {args.ranks_per_gpu} resident "
                                   f"traces, encode+decode round trip",
                       "job_ranks": args.world, "ranks_processed": ranks_done, "batches_per_gpu": len(plan),
                       "ranks_per_batch": args.ranks_per_gpu, "events_per_rank": args.events,
                       "records_per_step": int(total_records / args.steps),
                       "jitter": args.jitter, "rempi_max": args.max_len, "streams_per_gpu": n_lanes, "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                       "compressed_bytes_per_event": round(comp_per_event, 3),
                       "hbm_used_gb": round((total_b - free_b) / 1e9, 1), "hbm_total_gb": round(total_b / 1e9, 1),
                       "parallelism": f"dp{ws}: rank r -> GPU floor(r*{ws}/{args.world}), independent rank traces",
                       "verify": {"encode_ranks": int(counters[2]), "encode_failures": int(counters[3]),
                                  "decode_ranks": int(counters[4]), "decode_failures": int(counters[5]),
                                  "how": "decode: device-side round trip of every rank + reference SHA-256 of records/"
                                         "permutation for fixture ranks; encode: reference SHA-256 of the rank file "
                                         "for fixture ranks (+ CPU restatement bytes for --oracle-ranks)"},
                       "verify_failures": int(counters[3] + counters[5])},
            "roofline": {"bound": "hbm", "bound_note": "the fraction is against the HBM roofline as the contract asks; what limits "
                                                       "this kernel by itself is `limited_by` (vector-instruction issue: see "
                                                       "valu_issue_frac; latency: dependent steps of few waves)",
                         "limited_by": KERNEL_BOUND.get(dom, "hbm"), "kernel": dom, "achieved": dom_line["achieved"], "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": dom_line["frac"], "traffic": dom_line.get("traffic"),
                         "traffic_source": traffic.get("source") if traffic else None,
                         "launch_ms": round(launch_ms, 3),
                         "launch_ms_how": "HIP events, one lane alone on the GPU" if solo else
                                          "HIP events with all lanes in flight",
                         "launch_ms_concurrent": round(dom_ms / dom_launches, 3) if dom_launches else None,
                         "algorithmic_bytes_per_launch": dom_line["algorithmic_bytes_per_launch"],
                         "valu_issue_frac": dom_line.get("valu_issue_frac"),
                         "valu_issue_how": f"rocprofv3 SQ_INSTS_VALU per record x records x 4 cycles / ({SIMDS} SIMDs x "
                                           f"{SCLK_HZ / 1e9} GHz) / launch time: the share of the launch its vector "
                                           "instructions need at the issue rate of one per 4 cycles per SIMD",
                         "kernels": top,
                         "mix": {"matched_per_record": round(mix.m, 4), "pairs_per_matched": round(mix.pairs, 4),
                                 "compressed_bytes_per_record": round(mix.c, 3)},
                         "pipeline_achieved": round(pipeline_bytes(mix) * total_records / tmax / 1e9, 2),
                         "pipeline_algorithmic_bytes_per_record": round(pipeline_bytes(mix), 2),
                         "pipeline_traffic_per_record": None if traffic is None else traffic.get("pipeline_bytes_per_record"),
                         "pipeline_valu_per_record": None if traffic is None else traffic.get("pipeline_valu_per_record")},
            "cpu_baseline": cpu,
            "host_io": host_io,
            "configs": {"config2": cfg2},
        }
        print(json.dumps(out))
    for ln in lanes:
        ln.close()
    if dist:
        dist.destroy_process_group()


# Algorithmic HBM bytes per input record for each kernel, from the
# run's own mix: m = matched events per record, p = (id, delay) pairs per matched event, c =
# compressed bytes per record.  The dominant kernel's figure is the roofline numerator.
class Mix:
    def __init__(self, m, pairs, c):
        self.m, self.pairs, self.c = float(m), float(pairs), float(c)


# what limits each kernel alone on the GPU: "hbm" (streams its arrays), "valu" (vector-instruction
# issue: valu_issue_frac near 1), "latency" (a chain of dependent steps -- LDS or memory round
# trips -- on the waves its LDS or its unit count allow; the permutation rebuild got 23 % shorter
# from a smaller LDS footprint and 8 % from a quarter fewer vector instructions)
KERNEL_BOUND = {
    "k_tile_hist": "hbm", "k_scatter": "hbm", "k_unit_prep": "hbm", "k_window_rank": "valu", "k_sort_tiles": "lds",
    "k_rank_tiles": "lds", "k_epoch": "lds", "k_cuts": "hbm", "k_chain_grp8": "valu", "k_chain_grp16": "valu",
    "k_chain_grp64": "latency", "k_chain_seg": "latency", "k_chain_exits": "latency", "k_chain_mark": "latency",
    "k_positions": "hbm", "k_deltas": "valu", "k_write_units": "hbm", "k_chunks": "latency", "k_lists": "latency",
    "k_dec_sections": "hbm", "k_dec_pair_scan": "latency", "k_dec_perm_seg": "latency", "k_dec_perm_grp": "latency",
    "k_dec_perm_check": "hbm", "k_dec_records": "hbm",
}


def algorithmic_bytes(kernel, n_records, mix):
    m, p, c = mix.m, mix.pairs, mix.c
    per = {
        "k_tile_hist": 32,
        "k_scatter": 32 + 16 + 4,
        "k_unit_prep": 16 + m * (8 + 4),
        "k_window_rank": m * (8 + 4 + 4 + 8),
        "k_sort_tiles": m * (8 + 8 + 4),
        "k_rank_tiles": m * (8 + 4 + 8 + 4 + 4 + 8),
        "k_epoch": m * 8,
        "k_chain_grp8": m * (4 + 4 + 4),
        "k_chain_grp16": m * (4 + 4 + 4),
        "k_chain_mark": m * (4 + 1),
        "k_positions": m * (4 + 1 + 4 + (1 + p) + 4 + 1 + 4 + (1 + p) + (1 + p) * 8) / 2,  # mean of its two launches (rows, columns)
        "k_deltas": m * (2 * p * 4 + p * (4 + 4 + 4)),
        "k_write_units": m * (4 + 4 + 8) + c,
        "k_dec_sections": 0.3 * c,
        # the pair sections once (8 B per pair), perm and its inverse once each (4 + 4 B per matched event)
        "k_dec_perm_seg": m * (p * 8 + 8),
        "k_dec_perm_grp": m * (p * 8 + 8),
        "k_dec_pair_scan": m * p * 8,
        "k_dec_records": c + m * (4 + 8 + 8 + 1) + 32,
        "k_chain_exits": m * 4 * 0.4,   # the parents on the paths from each segment's max-level rows to its first row
        "k_cuts": m * (4 + 4),
    }.get(kernel)
    return None if per is None else per * n_records


PMC_TRAFFIC = "profiles/r03/pmc_traffic.json"


def pmc_traffic():
    """HBM bytes per record of every kernel from the committed rocprofv3 FETCH_SIZE / WRITE_SIZE
    passes (tools/pmc_traffic.py); None if not collected."""
    for rel in (PMC_TRAFFIC, "profiles/r02/pmc_traffic.json", "profiles/r01/pmc_traffic.json"):
        try:
            d = json.load(open(os.path.join(ROOT, rel)))
            d.setdefault("kernels", {})
            d["source"] = rel
            return d
        except (OSError, ValueError):
            continue
    return None


def pipeline_bytes(mix):
    """Algorithmic bytes of the whole path per record: encode reads 32 B/event and writes c;
    decode reads c + 8m of sorted keys and writes 32 B/event."""
    return 64 + 2 * mix.c + 8 * mix.m


if __name__ == "__main__":
    if len(sys.argv) == 4 and sys.argv[1] == "--port-one":
        port_one(sys.argv[2], int(sys.argv[3]))
    else:
        main()
