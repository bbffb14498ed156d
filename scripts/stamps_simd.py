#!/usr/bin/env python3
"""Per-SIMD issue occupancy of one chunk_hash launch from the raw per-wave stamps that
scripts/hash_stamps.py saves (STAMPS_OUT): for every SIMD, the share of the launch during which it
holds 0, 1, 2, 3 or 4 resident waves.  A SIMD issues at its full rate from two waves up (the
quarter-rate SHA mix: scripts/valu_issue_mb.hip), at about half with one wave, not at all with
none; so the tail's cost is the idle and one-wave SIMD time, weighted by those rates.

  python scripts/stamps_simd.py stamps_raw.npy [ceiling_gbps]"""
import json
import sys

import numpy as np


def main():
    a = np.load(sys.argv[1]).astype(np.uint64)
    r0, c0, r1, c1 = (a[:, k].astype(np.float64) for k in range(4))
    hw = a[:, 4]
    simd = ((hw >> 4) & 3).astype(np.int64)
    cu = ((hw >> 8) & 15).astype(np.int64)
    sh = ((hw >> 12) & 1).astype(np.int64)
    se = ((hw >> 13) & 7).astype(np.int64)
    xcc = ((hw >> 32) & 15).astype(np.int64)
    key = (((xcc * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd
    t0, t1 = r0.min(), r1.max()
    span = t1 - t0
    hist = np.zeros(9)
    simds = np.unique(key)
    for k in simds:
        m = key == k
        ev = np.concatenate([np.stack([r0[m], np.ones(m.sum())], 1), np.stack([r1[m], -np.ones(m.sum())], 1),
                             [[t0, 0.0], [t1, 0.0]]])
        ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
        occ = np.cumsum(ev[:, 1])
        dt = np.diff(ev[:, 0], append=t1)
        for w in range(9):
            hist[w] += dt[occ == w].sum()
    hist /= span * len(simds)
    # issue capacity relative to a SIMD with >= 2 waves all launch long: 0 waves -> 0, 1 wave -> ~0.5
    # (one wave issues an instruction per ~5 cycles, two or more per ~2.4-4.3)
    cap = hist[1] * 0.5 + hist[2:].sum()
    out = {"simds": int(len(simds)), "span_ms": round(span / 100e3, 4),
           "simd_time_frac_by_waves": {str(w): round(float(hist[w]), 4) for w in range(9) if hist[w] > 0},
           "issue_capacity_frac": round(float(cap), 4),
           "tail_loss": round(float(1 - cap), 4),
           "clock_mhz": round(float((c1 - c0).sum() / (r1 - r0).sum() * 100.0), 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
