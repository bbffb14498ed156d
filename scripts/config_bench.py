#!/usr/bin/env python3
"""The other BASELINE.json configurations on one MI355X, device-resident (bench.py is configs[1]).

CONFIG=dedup  (configs[2]): 8 GiB = 32768 write buffers of 256 KiB, 50 % of them byte copies of
              an earlier fresh buffer (seeded Bernoulli).  One step = the
              whole device write path of SparseDedupFile.writeCache for the batch: getChunks
              (CDC + SHA-256), the dedup-hit index (fresh per step), and the SparseDataChunk
              map images; LZ4 of the new chunks is timed beside it (on for compressed volumes).
CONFIG=backup (configs[4], one GPU's slice): BACKUP_VOLUME=true: 102 write buffers of 40 MiB
              (3.98 GiB), maxLen 128 KiB, tar-like stream (sdfs_amd.device.tar_layout: 512-byte
              headers, file bodies of log-uniform length zero-padded to 512, 20 % of bodies
              repeating an earlier one); one step = getChunks + the index + LZ4 of the new chunks
              (backup volumes compress).
Stage times are HIP events on the launch stream, averaged over STEPS steps.  One JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from sdfs_amd import HipVariableSha256HashEngine, SdfsConfig  # noqa: E402
from sdfs_amd.device import DeviceBatch  # noqa: E402
from sdfs_amd.index import HipHashesMap  # noqa: E402
from sdfs_amd.lz4 import HipLz4Compressor  # noqa: E402
from sdfs_amd.meta import emit_map_slots  # noqa: E402

CONFIG = os.environ.get("CONFIG", "dedup")
STEPS = int(os.environ.get("STEPS", "5"))


def fill_dedup(batch, nbuf, L, rng):
    batch.fill_streams(first_stream=0, bufs_per_stream=256)
    v = batch.data.view(nbuf, L)
    fresh = [0]
    src = np.arange(nbuf)
    for b in range(1, nbuf):
        if rng.random() < 0.5:
            fresh.append(b)
        else:
            src[b] = fresh[int(rng.integers(0, len(fresh)))]
    idx = torch.from_numpy(src).to(batch.data.device)
    dups = int((src != np.arange(nbuf)).sum())
    v.copy_(v.index_select(0, idx))  # copies of earlier fresh buffers (fresh ones map to themselves)
    return dups


def fill_backup(batch, total, rng):
    """The tar-like stream of configs[4] (sdfs_amd.device.tar_layout: 512-byte headers, log-uniform
    1 KiB-64 MiB bodies zero-padded to 512, 20 % of bodies repeating an earlier one), the same
    generator tests/test_gpu_parity.py::test_config4_tar_stream_per_gpu_share_16gib checks."""
    from sdfs_amd.device import tar_layout

    batch.fill_tar(tar_layout(total))
    torch.cuda.synchronize()


def main():
    rng = np.random.default_rng(0x5DF5)
    if CONFIG == "dedup":
        cfg = SdfsConfig()
        nbuf = int(os.environ.get("NBUF", "32768"))
    else:
        cfg = SdfsConfig.backup_volume()
        nbuf = int(os.environ.get("NBUF", "102"))
    L = cfg.chunk_length
    eng = HipVariableSha256HashEngine(config=cfg)
    batch = DeviceBatch(eng, nbuf=nbuf, buf_len=L)
    dup_bufs = fill_dedup(batch, nbuf, L, rng) if CONFIG == "dedup" else fill_backup(batch, nbuf * L, rng)
    torch.cuda.synchronize()
    cap = batch.nbuf * batch.cap
    ix = HipHashesMap(min(cap, 1 << 29))
    lz = HipLz4Compressor()
    s = torch.cuda.current_stream()
    ev = {k: [torch.cuda.Event(enable_timing=True) for _ in range(2)] for k in ("cdc", "index", "meta", "lz4")}
    acc = {k: 0.0 for k in ev}
    out = None

    def step(timed):
        nonlocal out
        ev["cdc"][0].record(s)
        batch.run(buffer_id_base=0, stream=s.cuda_stream)
        ev["cdc"][1].record(s)
        ev["index"][0].record(s)
        ix.clear(stream=s.cuda_stream)
        dup, loc, new, nc = ix.put_records(batch.recs.view(-1, 48), batch.total, pos_base=0, stream=s.cuda_stream)
        ev["index"][1].record(s)
        ev["meta"][0].record(s)
        m, doop, ovf = emit_map_slots(batch, dup, loc, stream=s.cuda_stream)
        ev["meta"][1].record(s)
        recs = batch.recs.view(-1, 48)
        ev["lz4"][0].record(s)
        so, sl, do, tot = lz.plan_records(recs, sel=new, count=nc.view(torch.int32), uniform_len=L,
                                          stream=s.cuda_stream)
        if out is None:
            room = batch.nbuf * L + batch.nbuf * L // 255 + 20 * cap + (1 << 20)  # >= sum of bound + 4
            out = torch.empty(room, dtype=torch.uint8, device=batch.data.device)
        dl = torch.empty(so.shape[0], dtype=torch.int32, device=batch.data.device)
        lz.compress_device(batch.data, so, sl, out, do, dl, count=nc.view(torch.int32), stream=s.cuda_stream)
        ev["lz4"][1].record(s)
        if timed:
            torch.cuda.synchronize()
            for k, (a, b) in ev.items():
                acc[k] += a.elapsed_time(b)
        return nc, dl, ovf, sl

    step(False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(STEPS):
        nc, dl, ovf, sl = step(True)
    wall = (time.perf_counter() - t0) / STEPS
    ms = {k: v / STEPS for k, v in acc.items()}
    nbytes = nbuf * L
    total = int(batch.total.item())
    new = int(nc.item())
    comp = int(dl[:new].to(torch.int64).sum().item())
    new_bytes = int(sl[:new].to(torch.int64).sum().item())
    gib = nbytes / 2**30
    res = {
        "bench": f"configs-{CONFIG}", "n_gpus": 1, "steps": STEPS, "input_gib": round(gib, 3),
        "chunks": total, "mean_chunk_bytes": round(nbytes / total, 1), "new_chunks": new,
        "dup_chunk_frac": round(1 - new / total, 4),
        "stage_ms": {k: round(v, 3) for k, v in ms.items()},
        "gibps": {
            "cdc_fingerprint": round(gib / (ms["cdc"] / 1e3), 1),
            "cdc_fingerprint_index": round(gib / ((ms["cdc"] + ms["index"]) / 1e3), 1),
            "cdc_fingerprint_index_map": round(gib / ((ms["cdc"] + ms["index"] + ms["meta"]) / 1e3), 1),
            "with_lz4_of_new_chunks": round(gib / (sum(ms.values()) / 1e3), 1),
        },
        "lz4_ratio_new_chunks": round(new_bytes / max(comp, 1), 3),
        "map_overflow": int(ovf.item()),
        "wall_ms_per_step_incl_event_syncs": round(wall * 1e3, 3),
    }
    if CONFIG == "dedup":
        res["duplicate_buffers"] = dup_bufs
    # per-kernel breakdown of the getChunks pipeline (HIP events around every kernel, untimed above)
    # and the chunk-length tail, which sets the fingerprint kernel's floor (one serial SHA-256
    # chain per chunk)
    eng.set_timing(STEPS)
    for _ in range(STEPS):
        batch.run(buffer_id_base=0, stream=s.cuda_stream)
    torch.cuda.synchronize()
    res["kernels_ms"] = {k: round(v, 4) for k, v in eng.kernel_times().items() if v}
    eng.set_timing(0)
    lens = batch.lens.view(batch.nbuf, batch.cap)
    valid = torch.arange(batch.cap, device=lens.device)[None, :] < batch.counts[:, None]
    cl = lens[valid].to(torch.int64)
    top = torch.topk(cl, min(8, cl.numel())).values.tolist()
    res["chunk_len"] = {"max": int(cl.max().item()), "top8": top,
                        "over_64KiB": int((cl > 65536).sum().item()), "over_32KiB": int((cl > 32768).sum().item())}
    # two batches in flight on two streams (two engines): batch i+1's scan overlaps the tail of
    # batch i's fingerprinting, where the longest chunks' serial SHA-256 leaves the GPU half idle
    eng2 = HipVariableSha256HashEngine(config=cfg)
    batch2 = DeviceBatch(eng2, nbuf=nbuf, buf_len=L)
    batch2.data = batch.data
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    pair = [batch, batch2]
    for k in range(2):
        pair[k].run(buffer_id_base=0, stream=streams[k].cuda_stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(2 * STEPS):
        pair[i % 2].run(buffer_id_base=0, stream=streams[i % 2].cuda_stream)
    torch.cuda.synchronize()
    two = (time.perf_counter() - t0) / (2 * STEPS)
    res["two_streams"] = {"ms_per_batch": round(two * 1e3, 3), "cdc_fingerprint_gibps": round(gib / two, 1),
                          "identical": bool(torch.equal(batch2.record_table(), batch.record_table()))}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
