#!/usr/bin/env python3
"""Host<->device copy rates on the box (pinned and pageable, 1 GiB), for the end-to-end path's
ceiling, and the engine's host batch at several staging sizes (max_batch_bytes)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from sdfs_amd import HipVariableSha256HashEngine, SdfsConfig  # noqa: E402

N = 1 << 30
d = torch.empty(N, dtype=torch.uint8, device="cuda")
pin = torch.empty(N, dtype=torch.uint8, pin_memory=True)
page = torch.empty(N, dtype=torch.uint8)
res = {}
for name, h in (("pinned", pin), ("pageable", page)):
    for direction in ("h2d", "d2h"):
        for _ in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if direction == "h2d":
                d.copy_(h, non_blocking=True)
            else:
                h.copy_(d, non_blocking=True)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
        res[f"{name}_{direction}_gbps"] = round(N / el / 1e9, 2)
print(json.dumps({"probe": "copy_rates_1GiB", **res}), flush=True)

L = 262144
nb = N // L
src = np.concatenate([np.random.default_rng(i).integers(0, 256, L, dtype=np.uint8) for i in range(64)])
for i in range(nb // 64):
    pin[i * 64 * L:(i + 1) * 64 * L].copy_(torch.from_numpy(src))
offs = np.arange(nb, dtype=np.uint64) * L
lens = np.full(nb, L, np.uint32)
page.copy_(pin)
for mb in (64, 256, 512):
    eng = HipVariableSha256HashEngine(config=SdfsConfig(max_batch_bytes=mb << 20))
    for name, host in (("pinned", pin.numpy()), ("pageable", page.numpy())):
        eng.chunk_batch(host, offs, lens)
        t0 = time.perf_counter()
        for _ in range(3):
            eng.chunk_batch(host, offs, lens)
        el = (time.perf_counter() - t0) / 3
        print(json.dumps({"probe": f"host_batch_{name}", "staging_mib": mb, "gibps": round(N / el / 2**30, 2)}),
              flush=True)
    eng.destroy()
