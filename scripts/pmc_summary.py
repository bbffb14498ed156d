#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (scripts/pmc_scan.sh) per kernel: mean counter value per
launch (after the first launches) and derived figures for the 4 GiB configs[1] batch:
instructions per input byte and per lane-byte, waits as fractions of wave cycles, effective
clock (GRBM_GUI_ACTIVE / 8 XCDs / kernel time).
usage: scripts/pmc_summary.py OUTDIR [--bytes 4294967296] [-o profiles/r02/pmc_summary.json]"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

KERNELS = {"cdc_scan_kernel": "cdc_scan", "chunk_hash_kernel": "chunk_hash", "lz4_lane_kernel": "lz4_lane",
           "lz4_compress_kernel": "lz4_wave", "lz4_decompress_lane_kernel": "lz4_dec_lane",
           "lz4_decompress_kernel": "lz4_dec_wave"}


def collect(d):
    per = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = next((v for n, v in KERNELS.items() if n in row["Kernel_Name"]), None)
            if k:
                per[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("outdir")
    ap.add_argument("--bytes", type=float, default=4294967296.0)
    ap.add_argument("--skip", type=int, default=2)
    ap.add_argument("-o", "--out")
    a = ap.parse_args()
    agg = defaultdict(dict)
    for sub in sorted(glob.glob(os.path.join(a.outdir, "*"))):
        if not os.path.isdir(sub):
            continue
        for k, cs in collect(sub).items():
            for c, v in cs.items():
                v = v[a.skip:] or v
                agg[k][c] = sum(v) / len(v)
    res = {}
    for k, c in agg.items():
        r = {"counters_mean_per_launch": {n: round(v, 1) for n, v in sorted(c.items())}}
        wave_bytes = a.bytes / 64.0  # one lane-byte per lane: a wave instruction covers 64 bytes
        if "SQ_INSTS_VALU" in c:
            r["valu_insts_per_wave_byte"] = round(c["SQ_INSTS_VALU"] / wave_bytes, 3)
        if "SQ_INSTS_LDS" in c:
            r["lds_insts_per_wave_byte"] = round(c["SQ_INSTS_LDS"] / wave_bytes, 3)
        if "SQ_INSTS_SALU" in c:
            r["salu_insts_per_wave_byte"] = round(c["SQ_INSTS_SALU"] / wave_bytes, 3)
        if "SQ_WAVE_CYCLES" in c:
            for w in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS",
                      "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
                if w in c:
                    r[f"{w}_frac_of_wave_cycles"] = round(c[w] / c["SQ_WAVE_CYCLES"], 3)
        res[k] = r
    print(json.dumps(res, indent=1))
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
