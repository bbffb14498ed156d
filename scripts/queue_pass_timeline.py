#!/usr/bin/env python3
"""Per-pass timeline of the coalescing queue from a rocprofv3 kernel + memory-copy trace
(scripts/probes/r6_qtrace.sh).  Every lane stream's operations in start order are cut into
passes (a pass ends with its fingerprint kernel; the first 40 % of each group, the warm-up, is
dropped); per group of lane streams: the pass span (H2D start -> fingerprint end), each
operation's median duration, the median gap before it, and how many passes' fingerprint kernels
run at once.  usage: queue_pass_timeline.py KERNEL_CSV MEMCOPY_CSV LABEL=S1,S2,... [...]"""
import csv
import json
import statistics as st
import sys
from collections import defaultdict


def kind(n):
    for k in ("copy_out", "prep_zero", "scan", "resolve", "prefix", "hash_split"):
        if k in n:
            return k
    return n[:20]


def main():
    ops = defaultdict(list)
    for r in csv.DictReader(open(sys.argv[1])):
        ops[int(r["Stream_Id"])].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind(r["Kernel_Name"])))
    for r in csv.DictReader(open(sys.argv[2])):
        if "HOST_TO_DEVICE" in r["Direction"]:
            ops[int(r["Stream_Id"])].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "H2D"))
    out = {}
    for spec in sys.argv[3:]:
        label, ids = spec.split("=")
        passes = []
        for s in (int(x) for x in ids.split(",")):
            cur = []
            for op in sorted(ops[s]):
                cur.append(op)
                if op[2] == "hash_split":
                    passes.append(cur)
                    cur = []
        passes = sorted(passes, key=lambda p: p[0][0])
        passes = passes[len(passes) * 2 // 5:]
        dur, gap, span = defaultdict(list), defaultdict(list), []
        for p in passes:
            span.append(p[-1][1] - p[0][0])
            for a, b in zip(p, p[1:]):
                gap[b[2]].append(b[0] - a[1])
            for o in p:
                dur[o[2]].append(o[1] - o[0])
        hs = [(o[0], o[1]) for p in passes for o in p if o[2] == "hash_split"]
        t0, t1 = min(a for a, _ in hs), max(b for _, b in hs)
        out[label] = {"passes": len(passes), "span_us_p50": round(st.median(span) / 1e3, 1),
                      "op_us_p50": {k: round(st.median(v) / 1e3, 1) for k, v in dur.items()},
                      "gap_before_us_p50": {k: round(st.median(v) / 1e3, 1) for k, v in gap.items()},
                      "fingerprint_kernels_in_flight": round(sum(b - a for a, b in hs) / (t1 - t0), 2)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
