#!/usr/bin/env python3
"""Does running one batch's scan beside another batch's fingerprinting pay on MI355X?

Two engines, two B1 batches (4 GiB each, same input), run back to back ITERS times either on one
stream (sequential) or on two streams (the GPU may overlap engine A's hash with engine B's scan).
HASH_VARIANTS picks the fingerprint kernel (sweep build: 6/7 = persistent grid of
SDFS_HASH_WG_PER_CU workgroups per CU, with / without block prefetch).  Prints GiB/s per mode."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ.setdefault("SDFS_CDC_LIB", os.path.join(ROOT, "sdfs_amd", "libsdfs_cdc_tuning.so"))

import torch  # noqa: E402

from sdfs_amd import HipVariableSha256HashEngine  # noqa: E402
from sdfs_amd.device import DeviceBatch  # noqa: E402

iters = int(os.environ.get("ITERS", "8"))
nbuf = int(os.environ.get("NBUF", "16384"))
configs = [c.split(":") for c in os.environ.get("CONFIGS", "0:0,6:1,6:2,6:3,7:2").split(",")]
data = None
ref = None
for hv, wpc in configs:
    os.environ["SDFS_HASH_VARIANT"] = hv
    os.environ["SDFS_HASH_WG_PER_CU"] = wpc
    engs = [HipVariableSha256HashEngine() for _ in range(2)]
    bats = [DeviceBatch(e, nbuf=nbuf, buf_len=262144) for e in engs]
    if data is None:
        bats[0].fill_streams(0, 256)
        data = bats[0].data
    for b in bats:
        b.data = data
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    res = {"hash_variant": int(hv), "wg_per_cu": int(wpc)}
    for mode in ("seq", "corun"):
        for rep in range(2):  # first pass warms up
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(iters):
                for k in range(2):
                    with torch.cuda.stream(streams[k] if mode == "corun" else streams[0]):
                        bats[k].run()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
        res[mode + "_gibps"] = round(2 * iters * nbuf * 262144 / dt / 2**30, 1)
        res[mode + "_ms_per_batch"] = round(dt / (2 * iters) * 1e3, 3)
    # results must not depend on the schedule
    c, st, ln, dg, tot = bats[1].host_results()
    if ref is None:
        ref = (c, st, ln, dg)
    res["identical"] = bool((c == ref[0]).all() and (st == ref[1]).all() and (ln == ref[2]).all()
                            and (dg == ref[3]).all())
    res["chunks"] = tot
    print(json.dumps(res), flush=True)
    del bats
    for e in engs:
        e.destroy()
