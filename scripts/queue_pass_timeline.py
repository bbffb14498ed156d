#!/usr/bin/env python3
"""Per-pass timeline of the coalescing queue from a rocprofv3 kernel + memory-copy trace
(scripts/probes/r6_qtrace.sh): for every lane stream, its operations in start order are cut into
passes (a pass ends with its copy_out kernel); per pass the H2D start -> copy_out end span, each
kernel's duration and the gaps between consecutive operations; medians per stream group, and how
many passes' fingerprint kernels overlap.  usage: queue_pass_timeline.py KERNEL_CSV MEMCOPY_CSV"""
import csv
import json
import statistics as st
import sys
from collections import defaultdict

KINDS = ("copy_out", "prep_zero", "scan", "resolve", "prefix", "scatter", "hash_split", "hash", "H2D")


def kind(name):
    for k in KINDS:
        if k in name:
            return k
    return name[:20]


def main():
    ops = defaultdict(list)
    for r in csv.DictReader(open(sys.argv[1])):
        ops[int(r["Stream_Id"])].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind(r["Kernel_Name"])))
    if len(sys.argv) > 2:
        for r in csv.DictReader(open(sys.argv[2])):
            if "HOST_TO_DEVICE" in r.get("Direction", "") + r.get("Operation", ""):
                sid = r.get("Stream_Id")
                if sid not in (None, "", "0"):
                    ops[int(sid)].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "H2D"))
    lanes = sorted(s for s, v in ops.items() if any(k == "copy_out" for _, _, k in v))
    passes = []
    for s in lanes:
        cur = []
        for op in sorted(ops[s]):
            cur.append(op)
            if op[2] == "copy_out":
                passes.append((s, cur))
                cur = []
    # group passes by caller-thread count: the probe runs one engine per thread count, so lanes are
    # new streams per group; split at the largest id gaps (six lanes per engine)
    groups = defaultdict(list)
    for s, p in passes:
        groups[(s - lanes[0]) // 6].append(p)
    out = {}
    for g, ps in sorted(groups.items()):
        span = [p[-1][1] - p[0][0] for p in ps]
        dur = defaultdict(list)
        gaps = []
        for p in ps:
            for a, b in zip(p, p[1:]):
                gaps.append(b[0] - a[1])
            for a in p:
                dur[a[2]].append(a[1] - a[0])
        hs = [(a[0], a[1]) for p in ps for a in p if a[2].startswith("hash")]
        t0 = min(a for a, _ in hs)
        t1 = max(b for _, b in hs)
        conc = sum(b - a for a, b in hs) / max(t1 - t0, 1)
        out[f"group{g}"] = {"passes": len(ps), "span_us_p50": round(st.median(span) / 1e3, 1),
                            "kernel_us_p50": {k: round(st.median(v) / 1e3, 1) for k, v in dur.items()},
                            "gap_us_p50": round(st.median(gaps) / 1e3, 1) if gaps else None,
                            "gap_us_sum_per_pass": round(sum(gaps) / len(ps) / 1e3, 1),
                            "hash_kernels_in_flight": round(conc, 2)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
