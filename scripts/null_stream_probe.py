#!/usr/bin/env python3
"""Read-path calls while the coalescing queue is busy: the queue's lanes are
blocking (CU-masked) streams, so any component call that used the legacy null stream waited for
every queue pass in flight.  Times single-block LZ4 decompress, the dedup index's getSize and a
single AES decrypt idle and while 48 threads call getChunks, p50/p99 in microseconds.

  SDFS_CDC_LIB=<library> python scripts/null_stream_probe.py [label]   (one JSON line)"""
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402,F401

from oracle import cdc_oracle as O  # noqa: E402  (synthetic data generator only)
from sdfs_amd import HipVariableSha256HashEngine  # noqa: E402
from sdfs_amd.index import HipHashesMap  # noqa: E402
from sdfs_amd.lz4 import HipLz4Compressor  # noqa: E402


def pct(xs):
    xs = sorted(xs)
    return {"p50_us": round(xs[len(xs) // 2] * 1e6, 1), "p99_us": round(xs[int(len(xs) * 0.99)] * 1e6, 1)}


def time_ops(fns, reps=200):
    out = {}
    for name, fn in fns.items():
        fn()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        out[name] = pct(ts)
    return out


def main():
    label = sys.argv[1] if len(sys.argv) > 1 else os.path.basename(os.environ.get("SDFS_CDC_LIB", "libsdfs_cdc.so"))
    eng = HipVariableSha256HashEngine()
    bufs = [O.synth(1, 500 + i, 0, 262144).tobytes() for i in range(64)]
    words = [b"alpha", b"beta", b"gamma", b"delta", b"chunk", b"store", b"write", b"buffer"]
    rng = np.random.default_rng(1)
    text = b" ".join(words[i] for i in rng.integers(0, len(words), 12000))[:65536]
    z = HipLz4Compressor()
    blk = z.compress(text)
    assert z.decompress(blk, len(text)) == text
    ix = HipHashesMap(1 << 16)
    fns = {"lz4_decompress_64k": lambda: z.decompress(blk, len(text)), "index_getSize": ix.getSize}
    idle = time_ops(fns)
    stop = threading.Event()
    calls = [0]

    def load(t):
        k = t
        while not stop.is_set():
            eng.chunk_arrays(bufs[k % len(bufs)])
            calls[0] += 1
            k += 48

    th = [threading.Thread(target=load, args=(t,), daemon=True) for t in range(48)]
    for t in th:
        t.start()
    time.sleep(1.0)
    c0, t0 = calls[0], time.perf_counter()
    busy = time_ops(fns)
    rate = (calls[0] - c0) * 262144 / (time.perf_counter() - t0) / 2**30
    stop.set()
    for t in th:
        t.join()
    print(json.dumps({"lib": label, "idle": idle, "busy_48_getchunks_threads": busy,
                      "getchunks_gibps_during": round(rate, 2)}), flush=True)
    z.destroy()
    ix.destroy()
    eng.destroy()


if __name__ == "__main__":
    main()
