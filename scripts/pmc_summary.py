#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc pass directories: mean counter value per launch of each named kernel
(the launches after the first `--skip` of that kernel, i.e. after warm-up).

usage: scripts/pmc_summary.py [--skip N] [--out JSON] PASS_DIR...
Each PASS_DIR holds one run's *_counter_collection.csv (any depth).  Kernels are keyed by the
short names of scripts/timeline.py (scan, hash, prefix, scatter, memset, ...)."""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
from collections import defaultdict

from timeline import short


def summarise(pass_dir: str, skip: int) -> dict:
    per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> value
    for f in glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                per[(short(r["Kernel_Name"]), int(r["Dispatch_Id"]))][r["Counter_Name"]] += float(r["Counter_Value"])
    out = defaultdict(dict)
    by_kernel = defaultdict(list)
    for (k, d), ctr in per.items():
        by_kernel[k].append((d, ctr))
    for k, rows in by_kernel.items():
        rows.sort()
        rows = rows[skip:] or rows
        for name in rows[0][1]:
            out[k][name] = sum(c[name] for _, c in rows) / len(rows)
        out[k]["launches"] = len(rows)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--skip", type=int, default=2)
    ap.add_argument("--out")
    a = ap.parse_args()
    res = {}
    for d in a.dirs:
        res[os.path.basename(os.path.normpath(d))] = summarise(d, a.skip)
    txt = json.dumps(res, indent=1, sort_keys=True)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
