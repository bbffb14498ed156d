#!/usr/bin/env python3
"""Clock and VALU-issue utilisation per kernel from one rocprofv3 run with --kernel-trace and
--pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU (scripts/profile_r4_end.sh, clock pass).

GRBM_GUI_ACTIVE is summed over the 8 XCDs and its window includes a fixed collection overhead
(the ~2 us memset dispatches read ~0.2 M cycles), taken off here as the median of the memset
dispatches.  clock = cycles per XCD / kernel duration; VALU utilisation = SQ_INSTS_VALU x 4 cycles
per wave64 instruction / (1 024 SIMDs x cycles per XCD).

usage: scripts/valu_clock.py RUN_DIR [--out JSON]"""
import argparse
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from timeline import short  # noqa: E402

XCDS, SIMDS = 8, 1024


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("run_dir")
    ap.add_argument("--out")
    ap.add_argument("--skip", type=int, default=2, help="warm-up dispatches of each kernel to skip")
    a = ap.parse_args()
    f = glob.glob(os.path.join(a.run_dir, "**", "*counter_collection.csv"), recursive=True)[0]
    per = defaultdict(dict)
    for r in csv.DictReader(open(f)):
        d = per[int(r["Dispatch_Id"])]
        d["kernel"] = short(r["Kernel_Name"])
        d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        d[r["Counter_Name"]] = float(r["Counter_Value"])
    over = statistics.median([d["GRBM_GUI_ACTIVE"] for d in per.values() if d["kernel"] == "memset"] or [0.0])
    by = defaultdict(list)
    for k in sorted(per):
        by[per[k]["kernel"]].append(per[k])
    out = {"source": os.path.relpath(f), "grbm_overhead_cycles_summed": over, "kernels": {}}
    for name, rows in by.items():
        rows = rows[a.skip:] or rows
        if name not in ("scan", "hash", "hash_long"):
            continue
        cyc = statistics.mean((r["GRBM_GUI_ACTIVE"] - over) / XCDS for r in rows)
        ns = statistics.mean(r["ns"] for r in rows)
        valu = statistics.mean(r["SQ_INSTS_VALU"] for r in rows)
        out["kernels"][name] = {"launches": len(rows), "duration_ms": ns / 1e6, "cycles_per_xcd": cyc,
                                "clock_ghz": cyc / ns, "sq_insts_valu": valu,
                                "valu_utilisation": valu * 4 / (SIMDS * cyc)}
    txt = json.dumps(out, indent=1)
    if a.out:
        open(a.out, "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
