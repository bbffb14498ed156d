#!/usr/bin/env python3
"""Scan-kernel variant sweep on the B1 workload (64 x 64 MiB, 256 KiB buffers) on one GPU.

For every (variant, segment length): times the pipeline with per-kernel HIP events and checks
that the chunk lists and digests are identical to variant 0's on the full 4 GiB.  Needs the
sweep build (make sweep).  Prints one JSON line per configuration."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("SDFS_CDC_LIB", os.path.join(ROOT, "sdfs_amd", "libsdfs_cdc_tuning.so"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from sdfs_amd import HipVariableSha256HashEngine  # noqa: E402
from sdfs_amd.device import DeviceBatch  # noqa: E402

variants = [int(v) for v in os.environ.get("VARIANTS", "0,1,2,3,4,5").split(",")]
segs = [int(v) for v in os.environ.get("SEGS", "4096").split(",")]
hvars = [int(v) for v in os.environ.get("HASH_VARIANTS", "0").split(",")]
steps = int(os.environ.get("STEPS", "5"))
nbuf = int(os.environ.get("NBUF", "16384"))
ref = None
data = None
for v, sl, hv in [(v, sl, hv) for v in variants for sl in segs for hv in hvars]:
    if True:
        os.environ["SDFS_HASH_VARIANT"] = str(hv)
        os.environ["SDFS_SCAN_VARIANT"] = str(v)
        os.environ["SDFS_SEG_LEN"] = str(sl)
        eng = HipVariableSha256HashEngine()
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
        counts, st, ln, dg, total = b.host_results()
        if ref is None:
            ref = (counts, st, ln, dg)
            same = True
        else:
            same = bool((counts == ref[0]).all() and (st == ref[1]).all() and (ln == ref[2]).all()
                        and (dg == ref[3]).all())
        nbytes = nbuf * 262144
        print(json.dumps(dict(variant=v, hash_variant=hv, seg_len=sl, scan_ms=round(kt["cdc_scan"], 4),
                              scan_gbps=round(nbytes / kt["cdc_scan"] / 1e6, 1),
                              hash_ms=round(kt["chunk_hash"], 4), resolve_ms=round(kt["cdc_resolve"], 4),
                              identical_to_v0=same, chunks=total)), flush=True)
        del b
        eng.destroy()
