#!/usr/bin/env python3
"""Backup profile (40 MiB write buffers): fingerprint-kernel time vs maxLen and hash variant.
Tests whether the longest chunk of a batch (a serial SHA-256 chain) sets the kernel's duration."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ.setdefault("SDFS_CDC_LIB", os.path.join(ROOT, "sdfs_amd", "libsdfs_cdc_tuning.so"))

import torch  # noqa: E402

from sdfs_amd import HipVariableSha256HashEngine, SdfsConfig  # noqa: E402
from sdfs_amd.device import DeviceBatch  # noqa: E402

data = None
for max_len in (32768, 65536, 131072):
    for hv in os.environ.get("HASH_VARIANTS", "0").split(","):
        os.environ["SDFS_HASH_VARIANT"] = hv
        e = HipVariableSha256HashEngine(config=SdfsConfig.backup_volume(max_len=max_len))
        b = DeviceBatch(e, nbuf=102, buf_len=40960 * 1024, records=False)
        if data is None:
            b.fill_streams(0, 1)
            data = b.data
        else:
            b.data = data
        b.run()
        torch.cuda.synchronize()
        e.set_timing(5)
        for _ in range(5):
            b.run()
        kt = e.kernel_times()
        e.set_timing(0)
        counts, st, ln, dg, total = b.host_results()
        print(json.dumps(dict(max_len=max_len, hash_variant=int(hv), chunks=total, longest=int(ln.max()),
                              hash_ms=round(kt["chunk_hash"], 3), scan_ms=round(kt["cdc_scan"], 3),
                              resolve_ms=round(kt["cdc_resolve"], 3))), flush=True)
        del b
        e.destroy()
