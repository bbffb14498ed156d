"""Multi-GPU sharding and the single fingerprint-table exchange.

Write streams are independent (every getChunks call starts from a fresh CDC state),
so whole streams are sharded across ranks with no data-path collective; the only exchange is ONE
all-gather of the per-rank fingerprint tables (48-byte records) so every GPU holds the global
fingerprint set (the input of the dedup-hit probe).  On ROCm the "nccl"
backend is RCCL over xGMI; the same code runs on "gloo" for CPU tests.

Protocol: all-gather the record counts (one int64 per rank), then all-gather the tables padded
to the largest count (all_gather_into_tensor needs equal sizes), then drop the padding.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

RECORD_BYTES = 48


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
