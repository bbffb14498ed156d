#!/usr/bin/env python3
"""Interleaved A/B of engine configurations in ONE process on the B1 workload (or BACKUP=1).

usage: CONFIGS="base:;pf:SDFS_HASH_VARIANT=4;seg8k:SDFS_SEG_LEN=8192" python3 scripts/ab.py
(MIN_SEG_KIB=2 MASK_BITS=11: the 4 KiB-mean chunk mix)
Each config is `name:ENV=VAL,ENV=VAL` (environment read by the engine at creation; the sweep
build is used by default so kernel variants can be selected).  The configurations run
round-robin ROUNDS times on the same device-resident input; per-stage device times are
reported as medians (and min) so box-to-box clock differences cancel out.  Results are also
checked identical across configurations."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("SDFS_CDC_LIB", os.path.join(ROOT, "sdfs_amd", "libsdfs_cdc_tuning.so"))

import torch  # noqa: E402

from sdfs_amd import HipVariableSha256HashEngine, SdfsConfig  # noqa: E402
from sdfs_amd.device import DeviceBatch  # noqa: E402

rounds = int(os.environ.get("ROUNDS", "10"))
backup = os.environ.get("BACKUP") == "1"
cfg = SdfsConfig.backup_volume() if backup else SdfsConfig()
if os.environ.get("MASK_BITS"):  # e.g. the 4 KiB-mean mix: MIN_SEG_KIB=2 MASK_BITS=11
    cfg = SdfsConfig(min_len=int(os.environ.get("MIN_SEG_KIB", "4")) * 1024 - 1,
                     pred_mask=(1 << int(os.environ["MASK_BITS"])) - 1)
buf_len = cfg.chunk_length
nbuf = int(os.environ.get("NBUF", "102" if backup else "16384"))
configs = []
for spec in os.environ.get("CONFIGS", "base:").split(";"):
    name, _, envs = spec.partition(":")
    env = dict(kv.split("=", 1) for kv in envs.split(",") if kv)
    configs.append((name, env))

engines, batches = [], []
data = None
for name, env in configs:
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    e = HipVariableSha256HashEngine(config=cfg)
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    b = DeviceBatch(e, nbuf=nbuf, buf_len=buf_len)
    if data is None:
        b.fill_streams(0, 1 if backup else 256)
        data = b.data
    else:
        b.data = data
    b.run()
    engines.append(e)
    batches.append(b)
torch.cuda.synchronize()

times = [dict() for _ in configs]
for r in range(rounds):
    for i, (e, b) in enumerate(zip(engines, batches)):
        e.set_timing(1)
        b.run()
        kt = e.kernel_times()
        e.set_timing(0)
        for k, v in kt.items():
            times[i].setdefault(k, []).append(v)

ref = None
for i, (name, env) in enumerate(configs):
    c, st, ln, dg, tot = batches[i].host_results()
    same = None
    if ref is None:
        ref = (c, st, ln, dg)
    else:
        same = bool((c == ref[0]).all() and (st == ref[1]).all() and (ln == ref[2]).all() and (dg == ref[3]).all())
    out = {"config": name, "env": env, "identical_to_first": same, "chunks": tot,
           "median_ms": {k: round(statistics.median(v), 4) for k, v in times[i].items() if max(v) > 0},
           "min_ms": {k: round(min(v), 4) for k, v in times[i].items() if max(v) > 0}}
    print(json.dumps(out), flush=True)
