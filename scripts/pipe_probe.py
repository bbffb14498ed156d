#!/usr/bin/env python3
"""Two batches in flight: does overlapping engine A's fingerprinting tail with engine B's scan pay
on the bench workload (BASELINE configs[1], 64 x 64 MiB, 4 GiB)?

  one      one engine, the whole 4 GiB batch per step, one stream (bench.py today)
  halves   two engines, each step = both 2 GiB halves of the batch on two streams
  alt      two engines, whole 4 GiB batches alternating on two streams (steady-state pipeline)
Records are checked identical to the one-engine run.  One JSON line per mode."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from sdfs_amd import HipVariableSha256HashEngine  # noqa: E402
from sdfs_amd.device import DeviceBatch  # noqa: E402

STEPS = int(os.environ.get("STEPS", "10"))
NBUF = 16384
L = 262144


def timed(fn, steps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def main():
    gib = NBUF * L / 2**30
    e0 = HipVariableSha256HashEngine()
    b0 = DeviceBatch(e0, nbuf=NBUF, buf_len=L)
    b0.fill_streams(first_stream=0, bufs_per_stream=256)
    s = [torch.cuda.Stream(), torch.cuda.Stream()]
    t = timed(lambda: b0.run(stream=s[0].cuda_stream), STEPS)
    ref = b0.record_table().clone()
    print(json.dumps({"mode": "one", "ms_per_4gib": round(t * 1e3, 3), "gibps": round(gib / t, 1)}), flush=True)

    # halves: two engines over the two halves of the same data
    e = [HipVariableSha256HashEngine() for _ in range(2)]
    h = [DeviceBatch(e[k], nbuf=NBUF // 2, buf_len=L) for k in range(2)]
    for k in range(2):
        h[k].data = b0.data[k * (NBUF // 2) * L:(k + 1) * (NBUF // 2) * L]

    def halves():
        for k in range(2):
            h[k].run(buffer_id_base=k * (NBUF // 2), stream=s[k].cuda_stream)

    t = timed(halves, STEPS)
    same = torch.equal(torch.cat([h[0].record_table(), h[1].record_table()], 0), ref)
    print(json.dumps({"mode": "halves", "ms_per_4gib": round(t * 1e3, 3), "gibps": round(gib / t, 1),
                      "identical": bool(same)}), flush=True)
    del h

    # alt: whole batches alternating
    b1 = DeviceBatch(e[0], nbuf=NBUF, buf_len=L)
    b1.data = b0.data
    pair = [b0, b1]
    i = [0]

    def alt():
        k = i[0] % 2
        pair[k].run(stream=s[k].cuda_stream)
        i[0] += 1

    t = timed(alt, 2 * STEPS)
    print(json.dumps({"mode": "alt", "ms_per_4gib": round(t * 1e3, 3), "gibps": round(gib / t, 1),
                      "identical": bool(torch.equal(b1.record_table(), ref))}), flush=True)


if __name__ == "__main__":
    main()
