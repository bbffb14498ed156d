#!/usr/bin/env python3
"""Fingerprint-kernel probe: chunk_hash time per byte as a function of the chunk-length mix.

Runs the B1 workload (64 x 64 MiB, 256 KiB buffers) with the production chunking parameters and
with forced uniform chunk lengths (min_len = L-1, max_len = L: every chunk is exactly L bytes
except the buffer tail), so the cost of length variance inside and across waves (and of the
kernel's tail) can be read off against a uniform schedule.  HASH_VARIANTS selects sweep-build
ablations (1 = no loads, 2 = no compression, 10 = 128-B-aligned loads); SHAPES filters the shapes.  One JSON line per configuration."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from sdfs_amd import HipVariableSha256HashEngine, SdfsConfig  # noqa: E402
from sdfs_amd.device import DeviceBatch  # noqa: E402

steps = int(os.environ.get("STEPS", "5"))
nbuf = int(os.environ.get("NBUF", "16384"))
hvars = [int(v) for v in os.environ.get("HASH_VARIANTS", "0").split(",")]
shapes = [("production", SdfsConfig())] + [
    (f"uniform{L}", SdfsConfig(min_len=L - 1, max_len=L)) for L in (4096, 8192, 16384, 32768)]
if os.environ.get("SHAPES"):
    shapes = [s for s in shapes if s[0] in os.environ["SHAPES"].split(",")]
data = None
for name, cfg in shapes:
    for hv in hvars:
        os.environ["SDFS_HASH_VARIANT"] = str(hv)
        eng = HipVariableSha256HashEngine(config=cfg)
        b = DeviceBatch(eng, nbuf=nbuf, buf_len=262144)
        if data is None:
            b.fill_streams(0, 256)
            data = b.data
        else:
            b.data = data
        b.run()
        torch.cuda.synchronize()
        eng.set_timing(steps)
        for _ in range(steps):
            b.run()
        kt = eng.kernel_times()
        eng.set_timing(0)
        total = int(b.total.item()) if hasattr(b, "total") else None
        nbytes = nbuf * 262144
        print(json.dumps(dict(shape=name, hash_variant=hv, hash_ms=round(kt["chunk_hash"], 4),
                              hash_gbps=round(nbytes / kt["chunk_hash"] / 1e6, 1),
                              scan_ms=round(kt["cdc_scan"], 4), chunks=total)), flush=True)
        del b
        eng.destroy()
