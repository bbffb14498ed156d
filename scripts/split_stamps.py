#!/usr/bin/env python3
"""Where the latency form of the fingerprint (chunk_hash_split_packed_kernel, the coalescing
queue's passes) spends a block: per-wave stamps of the producer wave (message schedule) and the
consumer wave (rounds), the cycles each spent waiting in the per-block barrier, and whether the
two waves of a group shared a SIMD.  A consumer that waits is held up by its producer.

  SDFS_CDC_LIB=sdfs_amd/libsdfs_cdc_tuning.so MASK_BITS=11 python scripts/split_stamps.py

One line per batch size (1 and 12 resident 256 KiB buffers: a lone caller's pass and a loaded
one), the stamps of REPS runs pooled."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from sdfs_amd import HipVariableSha256HashEngine, SdfsConfig, _lib  # noqa: E402
from sdfs_amd.device import DeviceBatch  # noqa: E402

REPS = int(os.environ.get("REPS", "32"))


def main():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    if not hasattr(lib, "sdfs_cdc_tuning_set_stamps"):
        raise SystemExit("needs SDFS_CDC_LIB=sdfs_amd/libsdfs_cdc_tuning.so")
    lib.sdfs_cdc_tuning_set_stamps.argtypes = [ctypes.c_void_p]
    mb = int(os.environ.get("MASK_BITS", "11"))
    cfg = SdfsConfig(min_len=2047, pred_mask=0x7FF) if mb == 11 else SdfsConfig()
    eng = HipVariableSha256HashEngine(config=cfg)
    for nbuf in (1, 12):
        b = DeviceBatch(eng, nbuf=nbuf, buf_len=262144)
        groups_max = nbuf * 160
        stamps = torch.zeros(groups_max * 2 * 8, dtype=torch.int64, device="cuda:0")
        rows = []
        for rep in range(REPS + 2):
            b.fill_streams(first_stream=1000 * rep, bufs_per_stream=1)
            lib.sdfs_cdc_tuning_set_stamps(stamps.data_ptr() if rep >= 2 else None)
            stamps.zero_()
            torch.cuda.synchronize()
            b.run()
            torch.cuda.synchronize()
            lib.sdfs_cdc_tuning_set_stamps(None)
            if rep < 2:
                continue
            a = stamps.view(-1, 8).cpu().numpy().astype(np.uint64)
            live = np.nonzero(a[:, 5] >> 32)[0]
            for g in sorted(set((live // 2).tolist())):
                p, c = a[2 * g], a[2 * g + 1]
                if (p[5] >> 32) == 0 or (c[5] >> 32) == 0:
                    continue
                nb = int(c[5] & 0xFFFFFFFF)
                hw_p, hw_c = int(p[4]), int(c[4])
                simd = lambda h: (h >> 32, (h >> 13) & 7, (h >> 8) & 15, (h >> 4) & 3)  # noqa: E731
                cu = lambda h: (h >> 32, (h >> 13) & 7, (h >> 8) & 15)  # noqa: E731
                rows.append({
                    "rep": rep, "group": g, "blocks": nb,
                    # per-block cycles over the first 32 blocks and over the rest (clock64 at block 32)
                    "early_cpb": (int(c[7] - c[1]) / 33) if nb > 64 and c[7] else None,
                    "late_cpb": (int(c[3] - c[7]) / (nb - 32)) if nb > 64 and c[7] else None,
                    "prod_cycles": int(p[3] - p[1]), "cons_cycles": int(c[3] - c[1]),
                    "prod_wait": int(p[6]), "cons_wait": int(c[6]),
                    "same_simd": simd(hw_p) == simd(hw_c), "cu": cu(hw_c),
                    "wall_ticks": int(c[2] - c[0]),
                })
        del b
        # the group that sets each run's time: its longest
        longest = {}
        for r in rows:
            if r["rep"] not in longest or r["blocks"] > longest[r["rep"]]["blocks"]:
                longest[r["rep"]] = r
        L = list(longest.values())
        cpb = [r["cons_cycles"] / (r["blocks"] + 1) for r in L]
        # groups sharing a CU within a run
        shared_cu = 0
        for rep in set(r["rep"] for r in rows):
            cus = [r["cu"] for r in rows if r["rep"] == rep]
            shared_cu += len(cus) - len(set(cus))
        # fixed cost vs per-block cost over every group: consumer cycles = F + c x (blocks + 1)
        X = np.array([r["blocks"] + 1 for r in rows], dtype=np.float64)
        Y = np.array([r["cons_cycles"] for r in rows], dtype=np.float64)
        c, F = np.polyfit(X, Y, 1) if len(rows) > 2 else (0.0, 0.0)
        if os.environ.get("STAMPS_OUT"):
            with open(os.environ["STAMPS_OUT"], "a") as f:
                for r in rows:
                    f.write(json.dumps(dict(r, cu=list(map(int, r["cu"])), mask_bits=mb, nbuf=nbuf, same_simd=bool(r["same_simd"]))) + "\n")
        print(json.dumps({
            "fit_cycles_per_block": round(float(c), 1), "fit_fixed_cycles": round(float(F), 0),
            "mask_bits": mb, "nbuf": nbuf, "groups": len(rows), "runs": len(L),
            "longest_group_blocks_median": float(np.median([r["blocks"] for r in L])),
            "cycles_per_block_median": round(float(np.median(cpb)), 1),
            "consumer_wait_frac": round(float(np.median([r["cons_wait"] / r["cons_cycles"] for r in L])), 4),
            "producer_wait_frac": round(float(np.median([r["prod_wait"] / r["prod_cycles"] for r in L])), 4),
            "all_groups_consumer_wait_frac": round(float(np.median([r["cons_wait"] / max(1, r["cons_cycles"]) for r in rows])), 4),
            "same_simd_frac": round(float(np.mean([r["same_simd"] for r in rows])), 4),
            "groups_sharing_a_cu": shared_cu,
            "shader_mhz": round(float(np.median([r["cons_cycles"] / r["wall_ticks"] * 100.0 for r in L])), 1),
        }), flush=True)
    eng.destroy()


if __name__ == "__main__":
    main()
