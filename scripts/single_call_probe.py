#!/usr/bin/env python3
"""Where one synchronous getChunks call of 256 KiB spends its time (VERDICT r4 next-round item 6:
SparseDedupFile.writeCache calls getChunks once per buffer and blocks, SparseDedupFile.java:432).

Per mix (the metric's 4 KiB mean and the reference default): (1) the device pipeline of ONE
resident 256 KiB buffer, per kernel (HIP events, sdfs_cdc_set_timing), with its longest chunk;
(2) the host entry the JNI glue uses (sdfs_cdc_get_chunks_fill), one caller, p50/p99 and the queue's
fill / copy / device split.  One JSON line per mix."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from sdfs_amd import HipVariableSha256HashEngine, SdfsConfig  # noqa: E402
from sdfs_amd import _lib  # noqa: E402
from sdfs_amd.device import DeviceBatch  # noqa: E402

REPS = int(os.environ.get("REPS", "64"))
for name, cfg in (("mix4k", SdfsConfig(min_len=2047, pred_mask=0x7FF)), ("default", SdfsConfig())):
    eng = HipVariableSha256HashEngine(config=cfg)
    b = DeviceBatch(eng, nbuf=1, buf_len=262144)
    rows = []
    for s in range(REPS):
        b.fill_streams(first_stream=7000 + s, bufs_per_stream=1)
        b.run()
        torch.cuda.synchronize()
        eng.set_timing(1)
        t0 = time.perf_counter()
        b.run()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e6
        kt = eng.kernel_times()
        eng.set_timing(0)
        counts, st, ln, dg, total = b.host_results()
        rows.append((wall, kt, int(ln[0, :counts[0]].max())))
    med = sorted(rows, key=lambda r: r[0])[len(rows) // 2]
    kmed = {k: round(float(np.median([r[1].get(k, 0.0) for r in rows])) * 1000.0, 1) for k in rows[0][1]}
    # host entry, one caller
    lat = []
    lib = _lib.load()
    cap = eng.slot_cap(262144)
    stv, lnv = np.zeros(cap, np.uint32), np.zeros(cap, np.uint32)
    dgv = np.zeros((cap, 32), np.uint8)
    n = ctypes.c_uint32()
    bufs = [np.frombuffer(np.random.default_rng(s).bytes(262144), np.uint8) for s in range(8)]
    for s in range(REPS * 2):
        src = bufs[s % 8]

        def _fill(ctx, dst, ln_, p=src.ctypes.data):
            ctypes.memmove(dst, p, ln_)
            return 0

        cb = _lib.FILL_FN(_fill)
        t0 = time.perf_counter()
        _lib.check(lib.sdfs_cdc_get_chunks_fill(eng._h, _lib.NO_STREAM, 262144, cb, None, stv.ctypes.data,
                                                lnv.ctypes.data, dgv.ctypes.data, cap, ctypes.byref(n)))
        lat.append((time.perf_counter() - t0) * 1e6)
    lat = np.array(lat[REPS // 2:])
    print(json.dumps({"mix": name, "device_one_buffer_us_median_wall": round(med[0], 1),
                      "device_kernels_us_median": kmed, "longest_chunk_median": int(np.median([r[2] for r in rows])),
                      "host_fill_entry": {"p50_us": round(float(np.percentile(lat, 50)), 1),
                                          "p99_us": round(float(np.percentile(lat, 99)), 1),
                                          "queue_split_us": eng.queue_timing()}}), flush=True)
    eng.destroy()
