#!/usr/bin/env python3
"""Coalescing-queue probe: T C threads calling getChunks (tools/threads_bench.c) on one engine;
prints rate, latency percentiles and the queue's own per-pass timeline (fill / copy / device).
Env: THREADS (list), QI (queue in-flight depths; tuning library only when != default),
CALLS_PER_THREAD (timed calls per thread, default 8: use >= 100 for A/B comparisons)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from sdfs_amd import HipVariableSha256HashEngine, SdfsConfig  # noqa: E402
from sdfs_amd.device import DeviceBatch  # noqa: E402
from tools import threads as T  # noqa: E402

L = 262144
nb = 1024
# MASK_BITS=11 MIN_SEG_KIB=2: the bench's 4 KiB-mean mix (default: the reference defaults)
MODE = os.environ.get("MODE", "copy")  # "fill": the JNI glue's entry (sdfs_cdc_get_chunks_fill)
cfg = SdfsConfig()
if os.environ.get("MASK_BITS"):
    cfg = SdfsConfig(min_len=int(os.environ.get("MIN_SEG_KIB", "4")) * 1024 - 1,
                     pred_mask=(1 << int(os.environ["MASK_BITS"])) - 1)
e0 = HipVariableSha256HashEngine(config=cfg)
b = DeviceBatch(e0, nbuf=nb, buf_len=L)
b.fill_streams(0, 64)
torch.cuda.synchronize()
host = b.data.cpu().numpy()
del b
e0.destroy()
def cpu_stat():
    """cgroup CPU throttling counters (cpu.stat): a quota-throttled process stalls for the rest of
    the period, which shows up as multi-millisecond outliers in the latency tail."""
    try:
        return {k: int(v) for k, v in (ln.split() for ln in open("/sys/fs/cgroup/cpu.stat"))}
    except Exception:
        return {}


def thread_cpu():
    """CPU seconds of this process's live threads by name (utime + stime): the queue's dispatcher
    and completers are named sdfs-qdisp / sdfs-qcomp (host_queue.h); the rest are the HIP/HSA
    runtime's threads and Python's."""
    tick = os.sysconf("SC_CLK_TCK")
    out = {}
    for t in os.listdir("/proc/self/task"):
        try:
            name = open(f"/proc/self/task/{t}/comm").read().strip()
            f = open(f"/proc/self/task/{t}/stat").read().rsplit(")", 1)[1].split()
            out[name] = out.get(name, 0.0) + (int(f[11]) + int(f[12])) / tick
        except OSError:
            pass
    return out


def proc_cpu():
    import resource
    r = resource.getrusage(resource.RUSAGE_SELF)
    return r.ru_utime + r.ru_stime


for th in [int(x) for x in os.environ.get("THREADS", "1,32,128,384").split(",")]:
    e = HipVariableSha256HashEngine(config=cfg)
    T.getchunks(e, th, host, L, max(256, 4 * th), mode=MODE)  # warm: every slot and lane carries a pass
    b0 = e.queue_stats()
    q0 = e.queue_early() if hasattr(e._lib, "sdfs_cdc_queue_early") else 0
    c0 = cpu_stat()
    t0, p0 = thread_cpu(), proc_cpu()
    calls = max(256, th * int(os.environ.get("CALLS_PER_THREAD", "8")))  # 8: a few ms per point (noisy)
    r, _ = T.getchunks(e, th, host, L, calls, mode=MODE)
    t1, p1 = thread_cpu(), proc_cpu()
    # host CPU per call (microseconds): the calling threads (measured in C), the queue's threads,
    # and everything else in the process (HIP runtime threads, Python)
    q = {k: t1[k] - t0.get(k, 0.0) for k in t1 if k.startswith("sdfs-q")}
    cpu = {"total": (p1 - p0) * 1e6 / calls, "callers": r.caller_cpu_us / calls, "fill_wall": r.fill_us / calls,
           "queue_threads": sum(q.values()) * 1e6 / calls}
    cpu["other"] = cpu["total"] - cpu["callers"] - cpu["queue_threads"]
    others = sorted(((t1[k] - t0.get(k, 0.0), k) for k in t1 if not k.startswith("sdfs-q")), reverse=True)[:3]
    cpu = {k: round(v, 1) for k, v in cpu.items()}
    cpu["top_other_threads_ms"] = {k: round(v * 1e3, 1) for v, k in others}
    if r.first_error:
        raise SystemExit(f"getChunks failed at {th} threads: status {r.first_error}")
    c1 = cpu_stat()
    b1 = e.queue_stats()
    early = (e.queue_early() - q0) if hasattr(e._lib, "sdfs_cdc_queue_early") else None
    thr = {k: c1[k] - c0.get(k, 0) for k in ("nr_throttled", "throttled_usec", "usage_usec") if k in c1}
    print(json.dumps({"threads": th, "qi": os.environ.get("SDFS_Q_INFLIGHT", "default"), "gibps": round(r.gibps, 3),
                      "p50_us": round(r.p50_us), "p99_us": round(r.p99_us), "early_calls": early,
                      "early_env": os.environ.get("SDFS_Q_EARLY", "default"), "mix": os.environ.get("MASK_BITS", "12"),
                      "calls_per_pass":
                      round((b1[1] - b0[1]) / max(b1[0] - b0[0], 1), 1), **e.queue_timing(), "cgroup": thr,
                      "cpu_us_per_call": cpu}),
          flush=True)
    e.destroy()
