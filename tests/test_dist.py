"""Multi-rank tests (gloo, world_size 2, 3 and 8 (the driver's scaling run), CPU): stream sharding and the fingerprint-table all-gather
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


def _exchange_worker(rank, world, port, q, direct=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cap = 12
        ex = RecordExchange(cap, "cpu", depth=2, slots=3 if direct else None)
        got = []
        table = torch.zeros(cap, RECORD_BYTES, dtype=torch.uint8)
        for step in range(5):
            n = (rank * 3 + step * 2) % (cap + 1)
            if direct:  # the producer writes into the exchange's own slot (bench.py's engine path)
                table = ex.acquire()
            table[:] = 255  # garbage beyond the count
            for i in range(n):
                table[i, :] = (step * 40 + rank * 10 + i) % 250
            ex.submit(table, torch.tensor([n]))
            if not direct:
                # the table is reused right away: the exchange must hold its own snapshot
                table[:] = 254
            if step == 2:
                got += ex.flush()
        got += ex.flush()
        q.put((rank, [(RecordExchange.compact(g, cl).numpy().tolist(), cl) for g, cl in got]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,direct", [(2, False), (3, False), (2, True), (3, True), (8, True)])
def test_record_exchange_pipelined_gloo(world, direct):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, q, direct)) for r in range(world)]
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


class _DictIndex:
    """CPU stand-in with HipHashesMap.put_records semantics (first copy in record order inserted at
    pos_base + its insertion rank, later copies dup with that position) for the gloo test."""

    def __init__(self):
        self.pos = {}

    def put_records(self, recs, count, pos_base=0):
        n = recs.shape[0]
        dup = torch.zeros(n, dtype=torch.uint8)
        loc = torch.zeros(n, dtype=torch.int64)
        for i in range(n):
            key = bytes(recs[i, :32].tolist())
            if key in self.pos:
                dup[i], loc[i] = 1, self.pos[key]
            else:
                self.pos[key] = pos_base + len(self.pos)
                loc[i] = self.pos[key]
        return dup, loc, None, None


def _shard_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sdfs_amd.dist import ShardedDedupIndex
        g = torch.Generator().manual_seed(7)
        pool = torch.randint(0, 256, (40, 32), generator=g, dtype=torch.uint8)  # shared fingerprints
        rg = torch.Generator().manual_seed(100 + rank)
        picks = torch.randint(0, 40, (25 + 5 * rank,), generator=rg)
        n = picks.shape[0]
        table = torch.zeros(max(40, n), RECORD_BYTES, dtype=torch.uint8)
        table[:n, :32] = pool[picks]
        table[:n, 32] = rank
        table[:n, 33] = torch.arange(n, dtype=torch.uint8)
        idx = ShardedDedupIndex(_DictIndex(), hash_len=32)
        dup, loc = idx.put_records(table, torch.tensor([n]))
        dup2, loc2 = idx.put_records(table, torch.tensor([n]))  # everything is known now
        q.put((rank, picks.tolist(), dup.tolist(), loc.tolist(), dup2.tolist(), loc2.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_sharded_dedup_index_gloo(world):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: rest for r, *rest in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    # reference: one global serial pass in (rank, record) order decides the first writer
    first = {}
    for r in range(world):
        for i, f in enumerate(res[r][0]):
            first.setdefault(f, (r, i))
    pos_of = {}
    for r in range(world):
        picks, dup, loc, dup2, loc2 = res[r]
        for i, f in enumerate(picks):
            assert dup[i] == (0 if first[f] == (r, i) else 1), (r, i)
            pos_of.setdefault(f, set()).add(loc[i])
            assert dup2[i] == 1 and loc2[i] == loc[i]
    assert all(len(v) == 1 for v in pos_of.values())  # one position per fingerprint, everywhere
    assert len({next(iter(v)) for v in pos_of.values()}) == len(pos_of)


def test_shard_of_matches_rocksdb_rule():
    from sdfs_amd.dist import shard_of
    recs = torch.zeros(256, RECORD_BYTES, dtype=torch.uint8)
    recs[:, 31] = torch.arange(256, dtype=torch.uint8)
    got = shard_of(recs, 8).tolist()
    for b in range(256):
        l = b - 256 if b >= 128 else b  # Java signed byte
        if l < 0:
            l = (l * -1) + 127
        assert got[b] == l // 32, b


# ---- configs[3] shape with CHUNKED records: every rank chunks its shard of the write streams
# (the oracle standing in for the engine on the CPU), builds the engine's 48-byte records
# {digest[32], u64 buffer_id, u32 start, u32 len} with bench.py's buffer ids (rank * nbuf + local),
# and exchanges them through RecordExchange (direct slots, 3 steps, as bench.py at N > 1).  Every
# rank must end with the global table in (rank, buffer, chunk) order, each step.
_S, _BPS, _BL = 2, 2, 65536  # streams per rank, buffers per stream and step, buffer length


def _rank_records(rank, world, step):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if root not in sys.path:
        sys.path.insert(0, root)
    from oracle import cdc_oracle as O
    streams = shard_streams(_S * world, world, rank)
    nbuf = len(streams) * _BPS
    out = bytearray()
    for k, s in enumerate(streams):
        for j in range(_BPS):
            data = O.synth_c(O.SYNTH_SEED, s, (step * _BPS + j) * _BL, _BL)
            st, ln, dg = O.chunk(data, O.Params())
            bid = rank * nbuf + k * _BPS + j
            for i in range(len(st)):
                out += dg[i].tobytes() + bid.to_bytes(8, "little") + int(st[i]).to_bytes(4, "little") + \
                    int(ln[i]).to_bytes(4, "little")
    return bytes(out)


def _chunked_exchange_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cap = _S * _BPS * (_BL // 4096 + 2)  # the engine's slot capacity bound per buffer, summed
        ex = RecordExchange(cap, "cpu", depth=2, slots=3)
        for step in range(3):
            recs = _rank_records(rank, world, step)
            n = len(recs) // RECORD_BYTES
            table = ex.acquire()
            table[:] = 255  # garbage beyond the count must not travel
            table[:n] = torch.frombuffer(bytearray(recs), dtype=torch.uint8).view(n, RECORD_BYTES)
            ex.submit(table, torch.tensor([n]))
        got = ex.flush()
        q.put((rank, [(RecordExchange.compact(g, cl).numpy().tobytes(), cl) for g, cl in got]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_configs3_chunked_records_exchange_gloo(world):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_chunked_exchange_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    nbuf = _S * _BPS
    for step in range(3):
        per_rank = [_rank_records(r, world, step) for r in range(world)]
        expect = b"".join(per_rank)
        for r in range(world):
            rows, counts = res[r][step]
            assert counts == [len(x) // RECORD_BYTES for x in per_rank]
            assert rows == expect, (r, step)
        # the gathered table covers every buffer of every rank exactly, in order
        recs = memoryview(expect)
        cover = {}
        for i in range(len(expect) // RECORD_BYTES):
            rec = recs[i * RECORD_BYTES:(i + 1) * RECORD_BYTES]
            bid = int.from_bytes(rec[32:40], "little")
            st = int.from_bytes(rec[40:44], "little")
            ln = int.from_bytes(rec[44:48], "little")
            assert st == cover.get(bid, 0)
            cover[bid] = st + ln
        assert cover == {b: _BL for b in range(world * nbuf)}


def _check_worker(rank, world, port, q):
    """bench.py's exchange self-check over a pipelined RecordExchange (direct slots), as the
    torchrun form at N > 1 runs it, with one rank's count deliberately off on the last step."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cap = 64
        ex = RecordExchange(cap, "cpu", depth=2, slots=3)
        ex.direct = True
        last = None
        for step in range(5):
            n = 10 + 3 * rank + step
            slot = ex.acquire()
            slot[:n] = (rank * 40 + step) % 256
            slot[n:] = 0xEE
            ex.submit(slot, torch.tensor([n]))
            last = (n, (ex.n - 1) % ex.nslots)
        res = ex.flush()
        (gathered, cl), k_last = res[-1], last[1]
        good = bench.exchange_check(torch, dist, gathered, cl, ex.slots[k_last], last[0], rank, world, "cpu")
        bad = bench.exchange_check(torch, dist, gathered, cl, ex.slots[k_last], last[0] + (rank == 1), rank, world, "cpu")
        q.put((rank, good, bad))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_bench_exchange_check_gloo(world):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_check_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, good, bad = q.get(timeout=180)
        res[r] = (good, bad)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for r, (good, bad) in res.items():
        assert good["counts"] == [10 + 3 * k + 4 for k in range(world)]
        assert good["counts_match"] and good["rows_match"]
        assert good["stride"] == max(good["counts"])
        assert (good["table_sha256"] is not None) == (r == 0)
        assert not bad["counts_match"] and bad["rows_match"]
