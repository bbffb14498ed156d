#!/usr/bin/env python3
"""Per-kernel L2->fabric read request sizes from a rocprofv3 counter pass of bench.py.

usage: scripts/pmc_reqsize.py DIR [-o OUT.json]

DIR is ``rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum
TCC_EA0_RDREQ_sum --output-format csv -d DIR``.  gfx950 splits the EA read requests by size
(32/64/128 B) and counts DRAM reads in 32-byte units (a 128-byte request counts 4), so the bytes
are exact here with no width calibration; they check the x2 correction applied to FETCH_SIZE
(which tallies every request as 64 B) by scripts/pmc_traffic.py.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
from collections import defaultdict

from pmc_traffic import STAGES


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("-o", default=None)
    a = ap.parse_args()
    vals = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            for sub, st in STAGES.items():
                if sub in r["Kernel_Name"]:
                    vals[st][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {"_note": "per launch, mean over launches after the first; bytes = 32 * TCC_EA0_RDREQ_DRAM_32B"}
    for st, cs in sorted(vals.items()):
        mean = {k: sum(v[1:]) / max(len(v) - 1, 1) for k, v in cs.items()}
        out[st] = {"launches": max(len(v) for v in cs.values()), **{k: round(v) for k, v in mean.items()},
                   "dram_read_bytes": round(32 * mean.get("TCC_EA0_RDREQ_DRAM_32B_sum", 0))}
    s = json.dumps(out, indent=1)
    print(s)
    if a.o:
        with open(a.o, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
