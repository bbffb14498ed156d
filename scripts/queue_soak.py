#!/usr/bin/env python3
"""Soak of the coalescing queue: for SOAK_SECS, C caller threads
(tools/threads_bench.c) hammer ONE shared engine with single-buffer getChunks calls at changing
thread counts while other C threads issue getHash calls on the same engine at the same time
(SDFS's flush threads and its getHash callers share the static engine,
SparseDedupFile.java:100,432; HashBlobArchive.java:1271).  Every kept result is compared with the
batch path's (getChunks) and with hashlib (getHash); any mismatch or error exits non-zero.
Random, all-zero (maxLen chunks: the longest SHA-256 chains) and short-period buffers are mixed.
usage: SOAK_SECS=60 python scripts/queue_soak.py"""
import hashlib
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from sdfs_amd import HipVariableSha256HashEngine  # noqa: E402
from tools import threads as T  # noqa: E402

L = 262144
NBUF = int(os.environ.get("NBUF", "512"))
SECS = float(os.environ.get("SOAK_SECS", "60"))
THREADS = [int(x) for x in os.environ.get("THREADS", "256,32,384,8,128,64").split(",")]


def main():
    rng = np.random.default_rng(0x50A4)
    data = rng.integers(0, 256, NBUF * L, dtype=np.uint8)
    v = data.reshape(NBUF, L)
    v[5::37] = 0                                            # all-zero buffers: maxLen chunks
    v[11::41] = np.tile(np.arange(61, dtype=np.uint8), L // 61 + 1)[:L]  # short period
    e = HipVariableSha256HashEngine()
    offs = np.arange(NBUF, dtype=np.uint64) * L
    counts, st, ln, dg = e.chunk_batch(data, offs, np.full(NBUF, L, np.uint32))
    # getHash callers: 8 KiB pieces of the same data, digests against hashlib
    HL = 8192
    hdata = data[: 4096 * HL]
    hexp = np.stack([np.frombuffer(hashlib.sha256(hdata[i * HL:(i + 1) * HL].tobytes()).digest(), np.uint8)
                     for i in range(4096)])
    errors = []
    stop = threading.Event()
    hash_calls = [0]

    def hasher():
        while not stop.is_set():
            r, dgs = T.gethash(e, 48, hdata, HL, 4096, keep=True)
            hash_calls[0] += int(r.calls)
            if r.first_error != 0:
                errors.append(f"getHash error {r.first_error}")
            elif not np.array_equal(dgs, hexp):
                errors.append(f"getHash mismatch in {int((dgs != hexp).any(axis=1).sum())} digests")

    th = threading.Thread(target=hasher, daemon=True)
    th.start()
    t0 = time.perf_counter()
    it, calls = 0, 0
    while time.perf_counter() - t0 < SECS and not errors:
        n = THREADS[it % len(THREADS)]
        r, (c2, s2, l2, d2) = T.getchunks(e, n, data, L, NBUF * 2, keep=True)
        calls += int(r.calls)
        bad = 0
        if r.first_error != 0:
            errors.append(f"getChunks error {r.first_error}")
        else:
            for b in range(NBUF):
                k = counts[b]
                if (c2[b] != k or not np.array_equal(s2[b, :k], st[b, :k]) or not np.array_equal(l2[b, :k], ln[b, :k])
                        or not np.array_equal(d2[b, :k], dg[b, :k])):
                    bad += 1
            if bad:
                errors.append(f"getChunks mismatch in {bad} buffers at {n} threads")
        print(json.dumps({"iter": it, "threads": n, "gibps": round(r.gibps, 2), "p99_us": round(r.p99_us, 1),
                          "calls": calls, "hash_calls": hash_calls[0], "bad_buffers": bad,
                          "elapsed_s": round(time.perf_counter() - t0, 1)}), flush=True)
        it += 1
    stop.set()
    th.join(120)
    passes, reqs = e.queue_stats()
    e.destroy()
    print(json.dumps({"soak_secs": round(time.perf_counter() - t0, 1), "getchunks_calls": calls,
                      "gethash_calls": hash_calls[0], "gpu_passes": passes, "requests": reqs,
                      "errors": errors}), flush=True)
    sys.exit(1 if errors else 0)


if __name__ == "__main__":
    main()
