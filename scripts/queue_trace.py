#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace of the coalescing-queue probe (scripts/probes/queue_trace_r5.sh):
per group of lane streams (one engine per caller-thread count), the median duration of each
pipeline kernel, how many passes' fingerprint kernels run at once (hash concurrency = summed
kernel time / wall span), and the median gap between a pass's fingerprint kernel and the next
operation on the same stream (the host round trip, when the result copy is issued after the
kernels).  usage: queue_trace.py KERNEL_TRACE_CSV [stream-group ...]  (group: comma-separated ids;
default: every stream that ran chunk_hash_split_kernel, grouped in fours by id)"""
import collections
import csv
import json
import statistics as st
import sys

KINDS = ('copy_out', 'copyBuffer', 'fillBuffer', 'scan', 'resolve', 'prefix', 'scatter', 'hash_split')


def kind(name):
    for k in KINDS:
        if k in name:
            return k
    return name[:24]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    if len(sys.argv) > 2:
        groups = [set(g.split(',')) for g in sys.argv[2:]]
    else:
        ids = sorted({int(r['Stream_Id']) for r in rows if 'hash_split' in r['Kernel_Name']})
        groups, cur = [], []
        for i in ids:
            if cur and i != cur[-1] + 1:
                groups.append({str(x) for x in cur})
                cur = []
            cur.append(i)
            if len(cur) == 4:
                groups.append({str(x) for x in cur})
                cur = []
        if cur:
            groups.append({str(x) for x in cur})
    for g in groups:
        rs = sorted((r for r in rows if r['Stream_Id'] in g), key=lambda r: int(r['Start_Timestamp']))
        if not rs:
            continue
        dur = collections.defaultdict(list)
        for r in rs:
            dur[kind(r['Kernel_Name'])].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
        hs = [(int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in rs if 'hash_split' in r['Kernel_Name']]
        span = (max(e for _, e in hs) - min(s for s, _ in hs)) / 1e3
        busy = sum(e - s for s, e in hs) / 1e3
        after = []
        by = collections.defaultdict(list)
        for r in rs:
            by[r['Stream_Id']].append(r)
        for lst in by.values():
            for a, b in zip(lst, lst[1:]):
                if 'hash_split' in a['Kernel_Name']:
                    after.append((int(b['Start_Timestamp']) - int(a['End_Timestamp'])) / 1e3)
        print(json.dumps({
            'streams': sorted(g, key=int), 'passes': len(hs),
            'kernel_us_median': {k: round(st.median(v), 1) for k, v in dur.items()},
            'hash_concurrency': round(busy / span, 2) if span else None,
            'after_hash_gap_us_median': round(st.median(after), 1) if after else None,
        }))


if __name__ == '__main__':
    main()
