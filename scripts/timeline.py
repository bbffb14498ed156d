#!/usr/bin/env python3
"""Timeline of a rocprofv3 kernel trace of bench.py's two-stream steps: where the device time of a
step goes.

usage: scripts/timeline.py KERNEL_TRACE_CSV [--first N] [--last M]

For the timed steps (kernels between dispatch --first and --last of the engine's pipeline) it
reports: the wall span, the busy fraction (any kernel running), the idle gaps, per-kernel mean
durations, how long each batch's fingerprint kernel waits after its scan ended (the small
prefix/scatter kernels and the memset in between), and how much of each fingerprint kernel runs
beside a scan of the other batch.
"""
from __future__ import annotations

import argparse
import csv
from collections import defaultdict

SHORT = {"cdc_scan_kernel": "scan", "chunk_hash_kernel": "hash", "cdc_prefix_kernel": "prefix",
         "cdc_scatter_kernel": "scatter", "fillBufferAligned": "memset", "seg_prefix_kernel": "seg_prefix",
         "cdc_resolve": "resolve", "chunk_hash_long_kernel": "hash_long"}


def short(name: str) -> str:
    for k, v in SHORT.items():
        if k in name:
            return v
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip-steps", type=int, default=5, help="pipeline runs to skip at the start")
    ap.add_argument("--steps", type=int, default=150, help="pipeline runs to analyse")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                         int(r["Queue_Id"]), int(r["Dispatch_Id"])))
    rows.sort()
    # a pipeline run = memset, scan, prefix, scatter, hash on one queue; key them by the scan
    scans = [r for r in rows if r[2] == "scan"]
    if len(scans) < a.skip_steps + a.steps:
        a.steps = max(1, len(scans) - a.skip_steps - 1)
    sel = scans[a.skip_steps: a.skip_steps + a.steps]
    t0, t1 = sel[0][0], sel[-1][1]
    win = [r for r in rows if r[0] >= t0 and r[1] <= t1 + 10_000_000]
    hashes = [r for r in win if r[2] == "hash"]
    # each scan's batch: the next hash on the same queue after it
    waits, overlaps, hash_durs = [], [], []
    for s in sel:
        h = next((x for x in rows if x[2] == "hash" and x[3] == s[3] and x[0] >= s[1]), None)
        if h is None:
            continue
        waits.append(h[0] - s[1])
        hash_durs.append(h[1] - h[0])
        ov = 0
        for o in scans:  # other batch's scans running beside this hash
            if o[3] != h[3]:
                ov += max(0, min(o[1], h[1]) - max(o[0], h[0]))
        overlaps.append(ov / max(1, h[1] - h[0]))
    end = max(r[1] for r in win if r[2] == "hash")
    span = end - t0
    # busy = union of kernel intervals
    iv = sorted((r[0], r[1]) for r in win if r[1] <= end)
    busy, cur_s, cur_e, gaps = 0, None, None, []
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    per = defaultdict(list)
    for r in win:
        per[r[2]].append(r[1] - r[0])
    n = len(sel)
    print(f"steps analysed: {n}, span {span / 1e6:.3f} ms = {span / n / 1e6:.4f} ms per step")
    print(f"busy (any kernel running): {busy / span:.4f}; idle gaps: {len(gaps)}, total "
          f"{sum(gaps) / 1e6:.3f} ms, largest {max(gaps) / 1e3 if gaps else 0:.1f} us")
    for k in ("memset", "scan", "prefix", "scatter", "hash"):
        if per[k]:
            v = per[k]
            print(f"  {k:8s} mean {sum(v) / len(v) / 1e6:.4f} ms  (n={len(v)})")
    if waits:
        print(f"scan end -> same batch's hash start: mean {sum(waits) / len(waits) / 1e6:.4f} ms, "
              f"max {max(waits) / 1e6:.4f} ms")
        print(f"hash duration: mean {sum(hash_durs) / len(hash_durs) / 1e6:.4f} ms; fraction of it beside "
              f"the other batch's scan: {sum(overlaps) / len(overlaps):.3f}")


if __name__ == "__main__":
    main()
