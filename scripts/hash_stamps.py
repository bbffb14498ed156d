#!/usr/bin/env python3
"""Where chunk_hash's remaining gap to its live VALU ceiling goes: clock,
tail and loads, on the BASELINE configs[1] batch at the metric's 4 KiB mix.

  SDFS_CDC_LIB=sdfs_amd/libsdfs_cdc_tuning.so python scripts/hash_stamps.py > stamps.json

* ceiling: the production sha256_compress register-only at 4 waves/SIMD on every CU (bench.py
  sha_ceiling) and its shader clock (tools/probe_kernels.hip sdfs_probe_sha256_clock);
* clock: fingerprint variant 50 = the production kernel with per-wave stamps (wall clock and shader
  clock at start and end, HW_ID/XCC_ID): the kernel's mean shader clock over its waves;
* tail: the wave-occupancy timeline from the stamps: mean resident waves / 4096 (4 per SIMD) over
  the launch, and the share of the launch with fewer than 4 waves per SIMD resident;
* loads: variant 45 = the production kernel without its data loads (message words from the state),
  its launch time against production's, same batch, same process.
The VALU fraction ~ clock ratio x occupancy x rest; `rest` is what neither explains (loads and
per-task overhead), cross-checked by the no-load ablation."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from sdfs_amd import HipVariableSha256HashEngine, SdfsConfig, _lib  # noqa: E402
from sdfs_amd.device import DeviceBatch  # noqa: E402

STEPS = 10


def run_variant(variant, stamps=None):
    os.environ["SDFS_HASH_VARIANT"] = str(variant)
    eng = HipVariableSha256HashEngine(config=SdfsConfig(min_len=2047, pred_mask=0x7FF))
    b = DeviceBatch(eng, nbuf=16384, buf_len=262144)
    b.fill_streams(first_stream=0, bufs_per_stream=256)
    for _ in range(3):
        b.run()
    torch.cuda.synchronize()
    eng.set_timing_stages(STEPS, ("chunk_hash",))
    for _ in range(STEPS):
        b.run()
    torch.cuda.synchronize()
    ms = eng.kernel_times().get("chunk_hash", 0.0)
    eng.set_timing(0)
    out = {"variant": variant, "chunk_hash_ms": round(ms, 4)}
    if stamps is not None:
        stamps.zero_()
        torch.cuda.synchronize()
        b.run()
        torch.cuda.synchronize()
        out["sha_blocks"] = bench.sha_blocks_of(torch, b)
    total = int(b.total.item())
    del b
    eng.destroy()
    return out, total


def main():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    if not hasattr(lib, "sdfs_cdc_tuning_set_stamps"):
        raise SystemExit("needs SDFS_CDC_LIB=sdfs_amd/libsdfs_cdc_tuning.so")
    khz = torch.cuda.get_device_properties(0)
    wall_mhz = 100.0
    try:
        hip = ctypes.CDLL("libamdhip64.so")
        v = ctypes.c_int()
        if hip.hipDeviceGetAttribute(ctypes.byref(v), 10017, 0) == 0 and v.value > 0:  # hipDeviceAttributeWallClockRate (kHz)
            wall_mhz = v.value / 1000.0
    except OSError:
        pass
    res = {"wall_clock_mhz": wall_mhz, "gpu": khz.name}
    # production and no-load ablation, interleaved twice
    prod, no_load = [], []
    for _ in range(2):
        prod.append(run_variant(0)[0]["chunk_hash_ms"])
        no_load.append(run_variant(45)[0]["chunk_hash_ms"])
    res["production_ms"] = prod
    res["no_loads_ms"] = no_load
    # stamped run
    nwaves = 16384 * 130 // 64 + 64
    stamps = torch.zeros(nwaves * 8, dtype=torch.int64, device="cuda:0")
    lib.sdfs_cdc_tuning_set_stamps.argtypes = [ctypes.c_void_p]
    lib.sdfs_cdc_tuning_set_stamps(stamps.data_ptr())
    st_run, total = run_variant(50, stamps)
    lib.sdfs_cdc_tuning_set_stamps(None)
    res["stamped"] = st_run
    a = stamps.view(-1, 8).cpu().numpy().astype(np.uint64)
    a = a[a[:, 0] != 0]
    if os.environ.get("STAMPS_OUT"):  # the raw per-wave stamps, for offline analysis
        np.save(os.environ["STAMPS_OUT"], a[:, :6])
    r0, c0, r1, c1 = (a[:, k].astype(np.float64) for k in range(4))
    t0, t1 = r0.min(), r1.max()
    span_ms = (t1 - t0) / wall_mhz / 1e3
    clock = (c1 - c0).sum() / (r1 - r0).sum() * wall_mhz
    # occupancy timeline: +1 at a wave's start, -1 at its end
    ev = np.concatenate([np.stack([r0, np.ones_like(r0)], 1), np.stack([r1, -np.ones_like(r1)], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    occ = np.cumsum(ev[:, 1])
    dt = np.diff(ev[:, 0], append=t1)
    full = 4096.0  # 256 CUs x 4 SIMDs x 4 waves (120 VGPRs)
    mean_occ = float((occ * dt).sum() / (t1 - t0))
    below = float(dt[occ < full].sum() / (t1 - t0))
    lost = float((np.clip(full - occ, 0, None) * dt).sum() / (full * (t1 - t0)))
    hw = a[:, 4]
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    se = (hw >> 13) & 7
    xcc = (hw >> 32) & 15
    res["waves"] = int(len(a))
    res["tasks"] = total
    res["span_ms_from_stamps"] = round(span_ms, 4)
    res["kernel_clock_mhz"] = round(float(clock), 1)
    res["mean_resident_waves"] = round(mean_occ, 1)
    res["occupancy_frac"] = round(mean_occ / full, 4)
    res["frac_of_launch_below_4_waves_per_simd"] = round(below, 4)
    res["lost_wave_slot_frac"] = round(lost, 4)
    res["distinct_simds"] = int(len(set(zip(xcc.tolist(), se.tolist(), cu.tolist(), simd.tolist()))))
    # tail shape: when the last 10 % / 1 % of waves end, as a fraction of the span
    ends = np.sort(r1)
    res["tail_last_waves_start_frac"] = {q: round(float((ends[int(len(ends) * (1 - q))] - t0) / (t1 - t0)), 4)
                                         for q in (0.10, 0.01)}
    # the ceiling and its clock, right after (same clock regime)
    res["ceiling_gbps"] = round(bench.sha_ceiling(0), 1)
    probe = ctypes.CDLL(bench.PROBE_LIB)
    mhz = ctypes.c_double()
    probe.sdfs_probe_sha256_clock.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
    rc = probe.sdfs_probe_sha256_clock(0, 4, 200, ctypes.byref(mhz))
    res["ceiling_clock_mhz"] = round(mhz.value, 1) if rc == 0 else None
    ms = float(np.median(prod))
    valu_gbps = st_run["sha_blocks"] * 64 / (ms / 1e3) / 1e9
    res["valu_frac"] = round(valu_gbps / res["ceiling_gbps"], 4)
    if res["ceiling_clock_mhz"]:
        clk = res["kernel_clock_mhz"] / res["ceiling_clock_mhz"]
        res["decomposition"] = {
            "clock_ratio": round(clk, 4),
            "occupancy": res["occupancy_frac"],
            "rest": round(res["valu_frac"] / (clk * res["occupancy_frac"]), 4),
            "no_load_speedup": round(float(np.median(prod) / np.median(no_load)), 4),
        }
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
