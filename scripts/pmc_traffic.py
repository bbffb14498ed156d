#!/usr/bin/env python3
"""Turn rocprofv3 FETCH_SIZE / WRITE_SIZE passes of bench.py into per-launch HBM bytes.

usage: scripts/pmc_traffic.py FETCH_DIR WRITE_DIR [-o profiles/pmc_traffic.json]

Each DIR is a ``rocprofv3 --pmc <counter> --output-format csv -d DIR`` output of the same bench
command (counters in separate passes: FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950).
Correction (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7): both counters are in KiB and
gfx950's FETCH_SIZE reports half the bytes of a wide streaming read, so
``hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024``.  The raw values are kept beside the result.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
from collections import defaultdict

# kernel-name substring -> stage name used by the engine's timing (sdfs_cdc_kernel_times)
STAGES = {
    "cdc_scan_kernel": "cdc_scan",
    "cdc_resolve_kernel": "cdc_resolve",
    "cdc_prefix_kernel": "cdc_prefix",
    "cdc_scatter_kernel": "cdc_scatter",
    "chunk_hash_kernel": "chunk_hash",
    "seg_prefix_kernel": "prep",
}


def read_counter(d: str, counter: str) -> dict:
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = defaultdict(list)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] != counter:
                    continue
                stage = next((v for k, v in STAGES.items() if k in row["Kernel_Name"]), None)
                if stage:
                    per[stage].append(float(row["Counter_Value"]))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("-o", "--out", default=os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                         "pmc_traffic.json"))
    ap.add_argument("--skip", type=int, default=1, help="launches to drop per kernel (warmup)")
    ap.add_argument("--params", default="", help="the bench's config.params string these passes measured")
    ap.add_argument("--source", default="", help="what was profiled (command / profile directory)")
    ap.add_argument("--commit", default="", help="git commit of the measured code")
    a = ap.parse_args()
    fetch = read_counter(a.fetch_dir, "FETCH_SIZE")
    write = read_counter(a.write_dir, "WRITE_SIZE")
    out = {"params": a.params, "source": a.source, "commit": a.commit}
    for stage in sorted(set(fetch) | set(write)):
        f = fetch.get(stage, [])[a.skip:] or fetch.get(stage, [])
        w = write.get(stage, [])[a.skip:] or write.get(stage, [])
        fk = sum(f) / len(f) if f else 0.0
        wk = sum(w) / len(w) if w else 0.0
        out[stage] = {
            "launches": [len(f), len(w)],
            "fetch_size_kib": round(fk, 1),
            "write_size_kib": round(wk, 1),
            "hbm_bytes_per_launch": int((2 * fk + wk) * 1024),
        }
    # one entry per measured chunk mix (the bench's params string), merged into the file
    try:
        doc = json.load(open(a.out))
    except Exception:
        doc = {}
    by = doc.get("by_params", {})
    if "params" in doc and doc["params"] not in by:  # the round-2 single-mix layout
        by[doc["params"]] = {k: v for k, v in doc.items() if k not in ("_note", "by_params")}
    by[a.params] = out
    doc = {"_note": "per chunk mix (bench.py config.params): hbm_bytes_per_launch = (2*FETCH_SIZE + "
                    "WRITE_SIZE) * 1024, mean over launches after warmup; FETCH_SIZE/WRITE_SIZE in KiB "
                    "(rocprofv3, gfx950 x2 read correction)", "by_params": by}
    with open(a.out, "w") as fh:
        json.dump(doc, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
