"""The N>1 path of bench.py on CPU: the job's ranks shard into one contiguous block per GPU
(rank r -> GPU floor(r G / R)) that together cover every rank exactly once, each GPU walks
its block in batches, nothing is exchanged on the data path, and the end-of-run reduction
(sum of counters, max of elapsed time) over a world_size-2 gloo group equals the
single-process totals over the whole job."""
import os

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_lib as O
import rempi_amd
from rempi_amd import shard


@pytest.mark.parametrize("world,gpus", [(1024, 1), (1024, 2), (1024, 4), (1024, 8), (1000, 8), (7, 8), (64, 3), (4096, 8)])
def test_blocks_cover_every_rank_exactly_once(world, gpus):
    shard.check_cover(world, gpus)
    seen = []
    for g in range(gpus):
        first, n = shard.block(world, gpus, g)
        seen += list(range(first, first + n))
        for r in range(first, first + n):
            assert shard.gpu_of_rank(r, world, gpus) == g
        bs = shard.batches(first, n, 96)
        assert [r for a, k in bs for r in range(a, a + k)] == list(range(first, first + n))
        assert all(0 < k <= 96 for _, k in bs)
    assert seen == list(range(world))


def test_config4_layout():
    """1024 ranks: 1 GPU walks 11 batches; 8 GPUs hold 128 ranks each as 64 + 64."""
    assert shard.block(1024, 1, 0) == (0, 1024)
    assert len(shard.batches(0, 1024, 96)) == 11
    assert shard.block(1024, 8, 7) == (896, 128)
    assert shard.batches(896, 128, 96) == [(896, 64), (960, 64)]
    assert shard.lane_sizes(10, 4) == [3, 3, 2, 2]
    assert shard.lane_sizes(3, 8) == [1, 1, 1]
    with pytest.raises(ValueError):
        shard.block(64, 2, 2)


WORLD = 10  # ranks of the toy job


def _worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    p = rempi_amd.default_gen_params(world_size=16, events_per_rank=3000)
    first, n = shard.block(WORLD, ws, rank)
    recs = comp = 0
    mine = []
    for a, k in shard.batches(first, n, 2):  # each process walks only its own block, batch by batch
        for r in range(a, a + k):
            h = rempi_amd.generate_host(p, r)
            recs += h.shape[0]
            comp += len(O.encode(h, 4096)[0])
            mine.append(r)
    c, t = shard.reduce_counters([recs, comp, len(mine), (1 << 53) + 1], 1.0 + rank, dist)
    q.put((rank, c.tolist(), t, mine))
    dist.destroy_process_group()


def test_gloo_world2_covers_the_whole_job():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in ps:
        pr.start()
    res = [q.get(timeout=240) for _ in ps]
    for pr in ps:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    p = rempi_amd.default_gen_params(world_size=16, events_per_rank=3000)
    recs = comp = 0
    for r in range(WORLD):
        h = rempi_amd.generate_host(p, r)
        recs += h.shape[0]
        comp += len(O.encode(h, 4096)[0])
    assert sorted(r for _, _, _, mine in res for r in mine) == list(range(WORLD))  # every rank once
    for _, c, t, _ in res:
        assert c == [recs, comp, WORLD, 2 * ((1 << 53) + 1)]  # (whole numbers, exact past 2^53)
        assert t == 2.0  # max over ranks
