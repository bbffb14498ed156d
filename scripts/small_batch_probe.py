#!/usr/bin/env python3
"""Device latency of SMALL batches (what one coalescing-queue pass costs): per-kernel HIP-event
times of run_device over nbuf = 1 .. 256 write buffers of 256 KiB, already in HBM, plus the
longest chunk of each batch (whose serial SHA-256 chain bounds chunk_hash).  One JSON line per
size.  Env: SIZES (list), REPS."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from sdfs_amd import HipVariableSha256HashEngine  # noqa: E402
from sdfs_amd.device import DeviceBatch  # noqa: E402

reps = int(os.environ.get("REPS", "20"))
eng = HipVariableSha256HashEngine()
for nb in [int(x) for x in os.environ.get("SIZES", "1,4,16,64,256").split(",")]:
    b = DeviceBatch(eng, nbuf=nb, buf_len=262144)
    b.fill_streams(first_stream=0, bufs_per_stream=max(1, min(nb, 256)))
    for _ in range(3):
        b.run()
    torch.cuda.synchronize()
    eng.set_timing(reps)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(reps):
        b.run()
    ev1.record()
    torch.cuda.synchronize()
    kt = eng.kernel_times()
    eng.set_timing(0)
    counts, st, ln, dg, total = b.host_results()
    longest = int(max(ln[i, :counts[i]].max() for i in range(nb)))
    print(json.dumps({"nbuf": nb, "ms_per_run": round(ev0.elapsed_time(ev1) / reps, 4),
                      "kernels_ms": {k: round(v, 4) for k, v in kt.items() if v}, "chunks": total,
                      "longest_chunk": longest, "longest_sha_blocks": (longest + 8) // 64 + 1}), flush=True)
    del b
eng.destroy()
