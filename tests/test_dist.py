"""Multi-rank tests (gloo, world_size 2, CPU): stream sharding and the fingerprint-table all-gather
that bench.py runs over RCCL at N>1 (sdfs_amd/dist.py)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from sdfs_amd.dist import RECORD_BYTES, RecordExchange, allgather_records, shard_streams


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        counts = [5, 0, 3, 7][:world]
        n = counts[rank]
        cap = 10
        table = torch.zeros(cap, RECORD_BYTES, dtype=torch.uint8)
        for i in range(n):
            table[i, :] = rank * 16 + i
        table[n:] = 255  # garbage beyond count must not travel
        out = allgather_records(table, n)
        q.put((rank, out.numpy().tolist()))
        # empty everywhere
        z = allgather_records(table, 0)
        assert z.shape == (0, RECORD_BYTES)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_allgather_records_gloo(world):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    counts = [5, 0, 3, 7][:world]
    expect = [[r * 16 + i] * RECORD_BYTES for r in range(world) for i in range(counts[r])]
    for r in range(world):
        assert res[r] == expect


def _exchange_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cap = 12
        ex = RecordExchange(cap, "cpu", depth=2)
        got = []
        table = torch.zeros(cap, RECORD_BYTES, dtype=torch.uint8)
        for step in range(5):
            n = (rank * 3 + step * 2) % (cap + 1)
            table[:] = 255  # garbage beyond the count
            for i in range(n):
                table[i, :] = (step * 40 + rank * 10 + i) % 250
            ex.submit(table, torch.tensor([n]))
            # the table is reused right away: the exchange must hold its own snapshot
            table[:] = 254
            if step == 2:
                got += ex.flush()
        got += ex.flush()
        q.put((rank, [(RecordExchange.compact(g, cl).numpy().tolist(), cl) for g, cl in got]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_record_exchange_pipelined_gloo(world):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for r in range(world):
        assert len(res[r]) == 5
        for step, (rows, cl) in enumerate(res[r]):
            ns = [(rr * 3 + step * 2) % 13 for rr in range(world)]
            assert cl == ns
            expect = [[(step * 40 + rr * 10 + i) % 250] * RECORD_BYTES for rr in range(world) for i in range(ns[rr])]
            assert rows == expect, (r, step)


def test_shard_streams_partition():
    for n, w in [(64, 1), (512, 8), (100, 3), (5, 8)]:
        parts = [shard_streams(n, w, r) for r in range(w)]
        flat = [s for p in parts for s in p]
        assert flat == list(range(n))
