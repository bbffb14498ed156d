#!/usr/bin/env python3
"""Round 4: what sets the backup profile's fingerprint time (configs[4] slice)?  The batch's chunk
extents are hashed through sdfs_cdc_hash_device (same fingerprint kernel, longest first) as they
are, with every chunk clipped to 32 KiB (the default maxLen), and the chunks > 32 KiB alone."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from config_bench import fill_backup  # noqa: E402
from sdfs_amd import HipVariableSha256HashEngine, SdfsConfig  # noqa: E402
from sdfs_amd.device import DeviceBatch  # noqa: E402

cfg = SdfsConfig.backup_volume()
eng = HipVariableSha256HashEngine(config=cfg)
L = cfg.chunk_length
b = DeviceBatch(eng, nbuf=102, buf_len=L)
fill_backup(b, 102 * L, np.random.default_rng(0x5DF5))
b.run()
torch.cuda.synchronize()
lens = b.lens.view(b.nbuf, b.cap)
valid = torch.arange(b.cap, device=lens.device)[None, :] < b.counts[:, None]
base = (torch.arange(b.nbuf, device=lens.device, dtype=torch.int64) * L)[:, None]
offs = (base + b.starts.view(b.nbuf, b.cap).to(torch.int64))[valid].contiguous()
ln = lens[valid].contiguous()
res = {"chunks": int(ln.numel())}


def timed(o, l, reps=10):
    dg = torch.empty(l.numel() * 32, dtype=torch.uint8, device=l.device)
    eng.hash_device(b.data, o, l, dg)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        eng.hash_device(b.data, o, l, dg)
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps, 4)


long = ln > 32768
res["as_is_ms"] = timed(offs, ln)
res["clipped_32k_ms"] = timed(offs, torch.clamp(ln, max=32768).contiguous())
res["long_only_ms"] = timed(offs[long].contiguous(), ln[long].contiguous())
res["long_count"] = int(long.sum().item())
res["max_len"] = int(ln.max().item())
res["bytes"] = int(ln.to(torch.int64).sum().item())
print(json.dumps(res), flush=True)
