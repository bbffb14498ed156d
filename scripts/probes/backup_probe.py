#!/usr/bin/env python3
"""Kernel split for the BACKUP_VOLUME profile (CHUNK_LENGTH 40 MiB, maxLen 128 KiB) on one GPU:
NBUF x 40 MiB synthetic buffers.  One JSON line with per-stage device milliseconds."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from sdfs_amd import HipVariableSha256HashEngine, SdfsConfig  # noqa: E402
from sdfs_amd.device import DeviceBatch  # noqa: E402

nbuf = int(os.environ.get("NBUF", "102"))
steps = int(os.environ.get("STEPS", "3"))
cfg = SdfsConfig.backup_volume()
eng = HipVariableSha256HashEngine(config=cfg)
b = DeviceBatch(eng, nbuf=nbuf, buf_len=cfg.chunk_length)
b.fill_streams(0, 1)
b.run()
torch.cuda.synchronize()
eng.set_timing(steps)
for _ in range(steps):
    b.run()
kt = eng.kernel_times()
tot = int(b.total.item())
nbytes = nbuf * cfg.chunk_length
print(json.dumps(dict(profile="backup", nbuf=nbuf, gib=round(nbytes / 2**30, 2), chunks=tot,
                      mean_chunk=round(nbytes / tot, 1), kernels_ms={k: round(v, 4) for k, v in kt.items()},
                      pipeline_gibps=round(nbytes / 2**30 / (kt["pipeline"] / 1e3), 1))), flush=True)
