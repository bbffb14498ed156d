"""Multi-GPU sharding and the single fingerprint-table exchange.

Write streams are independent (every getChunks call starts from a fresh CDC state),
so whole streams are sharded across ranks with no data-path collective; the only exchange is ONE
all-gather of the per-rank fingerprint tables (48-byte records) so every GPU holds the global
fingerprint set (the input of the dedup-hit probe).  On ROCm the "nccl"
backend is RCCL over xGMI; the same code runs on "gloo" for CPU tests.

Protocol: all-gather the record counts (one int64 per rank), then all-gather the tables padded
to the largest count (all_gather_into_tensor needs equal sizes), then drop the padding.

:class:`RecordExchange` runs that protocol pipelined for a stream of batches: batch i's table is
snapshotted on the producer stream and exchanged on a side stream while batch i+1 is being
chunked, so on N GPUs the exchange overlaps compute instead of adding to every step (SURVEY.md
8(e): ~24 MiB per GPU per step over xGMI).
"""
from __future__ import annotations

from collections import deque

import torch
import torch.distributed as dist

RECORD_BYTES = 48


def exchange_pg_options():
    """ProcessGroupNCCL options for the exchange's process group: RCCL's internal stream at high
    priority, so that its all-gather workgroups take CUs as soon as the chunking kernels free
    them instead of queueing behind them.  One-GPU projection of the 8-rank exchange (bench.py
    --exchange-proxy, profiles/r06/exchange_proxy/): +4 % per step instead of +21 % with the static
    scan stride, +2.5 % instead of +6 % with the work-queue scan.  None where the backend has no
    such options (gloo)."""
    try:
        from torch.distributed import ProcessGroupNCCL
    except ImportError:
        return None
    o = ProcessGroupNCCL.Options()
    o.is_high_priority_stream = True
    return o


def shard_streams(n_streams: int, world: int, rank: int) -> range:
    """Contiguous block of whole streams for `rank` (streams k*S/world .. (k+1)*S/world)."""
    lo = n_streams * rank // world
    hi = n_streams * (rank + 1) // world
    return range(lo, hi)


def allgather_records(table: torch.Tensor, count: int | torch.Tensor, group=None) -> torch.Tensor:
    """table: [>=count, 48] uint8 on this rank's device.  Returns [sum(counts), 48] in rank order."""
    world = dist.get_world_size(group)
    dev = table.device
    n = count if isinstance(count, torch.Tensor) else torch.tensor([count], device=dev)
    n = n.to(device=dev, dtype=torch.int64).reshape(1)
    counts = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(counts, n, group=group)
    cl = counts.tolist()
    mx = max(cl) if cl else 0
    if mx == 0:
        return table.new_empty((0, RECORD_BYTES))
    local = table[: cl[dist.get_rank(group)]]
    if local.shape[0] < mx:
        pad = table.new_zeros((mx - local.shape[0], RECORD_BYTES))
        local = torch.cat([local, pad], 0)
    gathered = table.new_empty((world * mx, RECORD_BYTES))
    dist.all_gather_into_tensor(gathered, local.contiguous(), group=group)
    parts = [gathered[r * mx: r * mx + cl[r]] for r in range(world)]
    return torch.cat(parts, 0)


class RecordExchange:
    """Pipelined all-gather of per-step fingerprint tables.

    ``submit(table, count)`` hands over step i's table and its device ``count`` on the producer
    stream (no host sync) and starts the count all-gather on a side stream; the table all-gather
    of a step is issued when ``depth`` steps are pending (or on ``flush``), after its counts are
    known on the side stream.  Tables live in a ring of ``slots`` buffers (default ``depth``).
    Two ways to fill a slot:

    * copy: ``submit`` snapshots ``table[:capacity]`` into the slot on the producer stream;
    * direct: ``acquire()`` returns the next slot for the engine to write its records into
      (``DeviceBatch.set_records``); ``submit`` of that same tensor copies nothing.  With
      ``slots > depth`` the slot's previous all-gather was issued a step earlier, so acquiring it
      never waits on the host — the producer stream only waits for that all-gather's event.

    Results are ``(gathered, counts)``: gathered is [world * max(counts), 48] in rank order, rank
    r's rows at [r * max, r * max + counts[r]).  On CPU tensors (gloo) every call is synchronous.
    """

    def __init__(self, capacity: int, device, group=None, depth: int = 2, slots: int | None = None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.capacity = int(capacity)
        self.depth = max(1, int(depth))
        self.nslots = max(self.depth, int(slots or self.depth))
        self.slots = [torch.empty(self.capacity, RECORD_BYTES, dtype=torch.uint8, device=self.device)
                      for _ in range(self.nslots)]
        self.cnt = [torch.zeros(1, dtype=torch.int64, device=self.device) for _ in range(self.nslots)]
        self.counts = [torch.zeros(self.world, dtype=torch.int64, device=self.device) for _ in range(self.nslots)]
        self.free = [None] * self.nslots  # side-stream event after a slot's table all-gather
        # counts reach the host through pinned memory + an event of their own: reading them must
        # not synchronise the whole side stream (that would wait for the newest step's production)
        self.counts_host = [torch.zeros(self.world, dtype=torch.int64, pin_memory=self.cuda)
                            for _ in range(self.nslots)]
        self.counts_ev = [None] * self.nslots
        self.side = torch.cuda.Stream(self.device, priority=-1) if self.cuda else None
        self.pending = deque()  # slots submitted, table all-gather not issued yet (oldest first)
        self.results = []
        self.n = 0
        self.direct = False  # callers that acquire() slots for the engine set this (bench.py)

    def _ctx(self):
        import contextlib
        return torch.cuda.stream(self.side) if self.cuda else contextlib.nullcontext()

    def _producer(self, stream):
        prod = stream if stream is not None else torch.cuda.current_stream(self.device)
        if not isinstance(prod, torch.cuda.Stream):
            prod = torch.cuda.ExternalStream(prod, device=self.device)
        return prod

    def _reclaim(self, slot: int, prod) -> None:
        """Make `slot` writable for the producer: issue its pending all-gather if it still has
        one (only when slots == depth), then order the producer after that all-gather."""
        while slot in self.pending:
            self.results.append(self._finish(self.pending.popleft()))
        if self.cuda and self.free[slot] is not None:
            prod.wait_event(self.free[slot])
            self.free[slot] = None

    def acquire(self, stream=None) -> torch.Tensor:
        """The slot the NEXT submit will exchange, free for the producer to write (see class doc)."""
        slot = self.n % self.nslots
        self._reclaim(slot, self._producer(stream) if self.cuda else None)
        return self.slots[slot]

    def submit(self, table: torch.Tensor, count, stream=None) -> None:
        # issue the oldest pending table all-gather BEFORE this step's count all-gather: torch's
        # process group runs its collectives in call order on one internal stream, and this step's
        # count exchange waits for this step's production
        while len(self.pending) >= self.depth:
            self.results.append(self._finish(self.pending.popleft()))
        slot = self.n % self.nslots
        self.n += 1
        prod = self._producer(stream) if self.cuda else None
        self._reclaim(slot, prod)
        # the acquired slot itself (the engine wrote its records in place): nothing to copy
        direct = table.data_ptr() == self.slots[slot].data_ptr()
        n = min(self.capacity, table.shape[0])
        c = count if isinstance(count, torch.Tensor) else torch.tensor([count], device=self.device)
        if self.cuda:
            with torch.cuda.stream(prod):
                if not direct:
                    self.slots[slot][:n].copy_(table[:n], non_blocking=True)
                self.cnt[slot].copy_(c.reshape(1).to(torch.int64), non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(prod)
            self.side.wait_event(ev)
        else:
            if not direct:
                self.slots[slot][:n].copy_(table[:n])
            self.cnt[slot].copy_(c.reshape(1).to(torch.int64))
        with self._ctx():
            dist.all_gather_into_tensor(self.counts[slot], self.cnt[slot], group=self.group)
            if self.cuda:
                self.counts_host[slot].copy_(self.counts[slot], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.side)
                self.counts_ev[slot] = ev
            else:
                self.counts_host[slot].copy_(self.counts[slot])
        self.pending.append(slot)

    def _finish(self, slot: int):
        with self._ctx():
            if self.cuda:
                self.counts_ev[slot].synchronize()  # this step's counts only
            cl = self.counts_host[slot].tolist()
            if max(cl) > self.capacity:
                raise ValueError(f"record count {max(cl)} exceeds the exchange capacity {self.capacity}")
            mx = max(cl) if cl else 0
            gathered = torch.empty(self.world * mx, RECORD_BYTES, dtype=torch.uint8, device=self.device)
            if mx:
                dist.all_gather_into_tensor(gathered, self.slots[slot][:mx], group=self.group)
            if self.cuda:
                ev = torch.cuda.Event()
                ev.record(self.side)
                self.free[slot] = ev
        return gathered, cl

    def flush(self) -> list:
        """Finish every pending step; returns (and clears) all results in submission order."""
        while self.pending:
            self.results.append(self._finish(self.pending.popleft()))
        out, self.results = self.results, []
        return out

    @staticmethod
    def compact(gathered: torch.Tensor, counts) -> torch.Tensor:
        """Drop the padding: [sum(counts), 48] in rank order."""
        mx = max(counts) if counts else 0
        return torch.cat([gathered[r * mx: r * mx + c] for r, c in enumerate(counts)], 0) if mx else \
            gathered.new_empty((0, RECORD_BYTES))


# ---- partitioned dedup-hit index across ranks (SURVEY.md 8(e) "alternative") ----------------

def shard_of(records: torch.Tensor, world: int, hash_len: int = 32) -> torch.Tensor:
    """Owner rank of each record's fingerprint: RocksDBMap's shard rule generalised to `world`
    shards (RocksDBMap.java:373-379 with dbs.length = 8: l = key[last] as a signed byte, l < 0 ->
    -l + 127, shard = l / 32); here shard = l * world / 256, identical to it at world = 8."""
    last = records[:, hash_len - 1].to(torch.int64)
    l = torch.where(last >= 128, (256 - last) + 127, last)  # signed byte b < 0 -> -b + 127
    return (l * world) // 256


class ShardedDedupIndex:
    """The dedup-hit index split across ranks by fingerprint: every rank owns one shard (its
    ``index``: a HipHashesMap, or any object with the same ``put_records``).

    ``put_records(table, count)`` — this rank's fingerprint records (e.g. its engine's record
    table) — routes every record to its owner with one all-to-all, applies them there in
    (source rank, record) order, and returns each record's ``(dup u8[n], hashloc int64[n])`` to
    its writer with a second all-to-all, in the caller's record order.  A fingerprint first
    written by several ranks in the same batch is inserted once: the lowest rank's copy wins and
    the others get ``dup = 1`` and its position.  Positions are ``pos_base + (rank << 40) + k``.
    """

    def __init__(self, index, group=None, hash_len: int = 32):
        self.index = index
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.hash_len = hash_len

    def put_records(self, table: torch.Tensor, count, pos_base: int = 0):
        dev = table.device
        n = int(count.item()) if isinstance(count, torch.Tensor) else int(count)
        recs = table[:n]
        owner = shard_of(recs, self.world, self.hash_len) if n else torch.zeros(0, dtype=torch.int64, device=dev)
        order = torch.argsort(owner, stable=True)
        send = recs[order].contiguous()
        send_counts = torch.bincount(owner, minlength=self.world).to(torch.int64)
        recv_counts = torch.empty_like(send_counts)
        dist.all_to_all_single(recv_counts, send_counts, group=self.group)
        sc, rc = send_counts.tolist(), recv_counts.tolist()
        recv = torch.empty(sum(rc), RECORD_BYTES, dtype=torch.uint8, device=dev)
        dist.all_to_all_single(recv, send, output_split_sizes=rc, input_split_sizes=sc, group=self.group)
        # apply in (source rank, record) order on this rank's shard
        m = recv.shape[0]
        if m:
            dup, loc, _, _ = self.index.put_records(recv, None, pos_base=pos_base + (self.rank << 40))
            dup, loc = dup[:m], loc[:m]
        else:
            dup = torch.zeros(0, dtype=torch.uint8, device=dev)
            loc = torch.zeros(0, dtype=torch.int64, device=dev)
        # results back to the writers, then into the caller's record order
        back_dup = torch.empty(n, dtype=torch.uint8, device=dev)
        back_loc = torch.empty(n, dtype=torch.int64, device=dev)
        dist.all_to_all_single(back_dup, dup.contiguous(), output_split_sizes=sc, input_split_sizes=rc,
                               group=self.group)
        dist.all_to_all_single(back_loc, loc.contiguous(), output_split_sizes=sc, input_split_sizes=rc,
                               group=self.group)
        out_dup = torch.empty_like(back_dup)
        out_loc = torch.empty_like(back_loc)
        out_dup[order] = back_dup
        out_loc[order] = back_loc
        return out_dup, out_loc


# ---- one process driving a device set (include/sdfs_cdc.h "Devices") ------------------------

class DeviceSetExchange:
    """The fingerprint-table exchange of ONE engine spanning several GPUs in one process: the
    engine all-gathers its devices' record tables itself, over RCCL (xGMI), with one communicator
    per device (``sdfs_cdc_allgather_records``) — the in-process counterpart of
    :class:`RecordExchange` (one rank per GPU over torch.distributed).

    Pipelined one step behind production: ``acquire(i, d, stream)`` hands device d the record slot
    of step i (a ring of ``slots``) and orders ``stream`` after that slot's previous exchange;
    ``produced(i, d, total, stream)`` marks step i's table on device d complete (an event on the
    producer stream); ``exchange(i)`` — called after step i+1 has been launched, so the devices
    stay busy — runs the exchange of step i on a side stream per device.  The call blocks only for
    step i's counts.  Results: ``(counts, stride)`` per step; gathered tables in ``gathered[d][i %
    2]`` (device j's rows at j * stride)."""

    def __init__(self, engine, capacity: int, devices, slots: int = 3):
        self.engine = engine
        self.devices = [torch.device(d) for d in devices]
        n = len(self.devices)
        self.capacity = int(capacity)
        self.nslots = slots
        self.slots = [[torch.empty(self.capacity, RECORD_BYTES, dtype=torch.uint8, device=dv) for _ in range(slots)]
                      for dv in self.devices]
        self.gathered = [[torch.empty(n * self.capacity, RECORD_BYTES, dtype=torch.uint8, device=dv) for _ in range(2)]
                         for dv in self.devices]
        # high priority: the exchange's RCCL workgroups take CUs as the chunking kernels free them
        # (exchange_pg_options)
        self.side = [torch.cuda.Stream(dv, priority=-1) for dv in self.devices]
        self.free = [[None] * slots for _ in self.devices]      # side-stream event: slot's exchange done
        self.prod = [[None] * slots for _ in self.devices]      # producer event: slot's table written
        self.totals = [[None] * slots for _ in self.devices]    # the step's device count tensor
        self.results = []

    def acquire(self, i: int, d: int, stream) -> torch.Tensor:
        k = i % self.nslots
        if self.free[d][k] is not None:
            stream.wait_event(self.free[d][k])
            self.free[d][k] = None
        return self.slots[d][k]

    def produced(self, i: int, d: int, total: torch.Tensor, stream) -> None:
        k = i % self.nslots
        ev = torch.cuda.Event()
        ev.record(stream)
        self.prod[d][k] = ev
        self.totals[d][k] = total

    def exchange(self, i: int):
        k = i % self.nslots
        for d, s in enumerate(self.side):
            s.wait_event(self.prod[d][k])
        res = self.engine.allgather_records([self.slots[d][k] for d in range(len(self.devices))],
                                            [self.totals[d][k] for d in range(len(self.devices))],
                                            [self.gathered[d][i % 2] for d in range(len(self.devices))],
                                            streams=[s.cuda_stream for s in self.side])
        for d, s in enumerate(self.side):
            ev = torch.cuda.Event()
            ev.record(s)
            self.free[d][k] = ev
        self.results.append(res)
        return res
