#!/usr/bin/env python3
"""LZ4 of unique chunks on one MI355X: device-resident GiB/s of input.

Workload: NBUF write buffers of 256 KiB (default 4096 = 1 GiB) chunked by the engine with the
reference parameters; every chunk is treated as new (0 % duplicates) and compressed into its
putChunk record ([BE length][LZ4 block], HashBlobArchive.java:1281-1289).  Two data sets:
`random` (the B1 synthetic streams: incompressible, the search skips ahead) and `text` (a
word-salad corpus, ~2.5x compressible: many short matches).  Reports the kernel's device time
(HIP events on the launch stream), GiB/s of input, the compression ratio, and the CPU oracle
(oracle/lz4_ref.c, the same parse) on a sample of the same chunks with THREADS host threads.
One JSON line per data set and mode."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import cdc_oracle as C  # noqa: E402  (CPU baseline and spot checks only)
from oracle import lz4_oracle as Z  # noqa: E402
from sdfs_amd import HipVariableSha256HashEngine  # noqa: E402
from sdfs_amd.device import DeviceBatch  # noqa: E402
from sdfs_amd.lz4 import HipLz4Compressor  # noqa: E402

NBUF = int(os.environ.get("NBUF", "4096"))
REPS = int(os.environ.get("REPS", "5"))
THREADS = int(os.environ.get("THREADS", "16"))
CPU_SECS = float(os.environ.get("CPU_SECS", "8"))
MODES = [m for m in os.environ.get("MODES", "r123,v19").split(",") if m]
SETS = [s for s in os.environ.get("SETS", "random,text").split(",") if s]
L = 262144


def text_corpus(nbytes: int) -> np.ndarray:
    """Vectorised word salad (the vocabulary of oracle/lz4_oracle.text_like), 64 MiB tiled."""
    words = [w + b" " for w in Z._WORDS]
    vocab = np.frombuffer(b"".join(words), np.uint8)
    wl = np.array([len(w) for w in words])
    wo = np.concatenate([[0], np.cumsum(wl)[:-1]])
    base_n = min(nbytes, 64 << 20)
    nw = base_n // 3 + 16
    idx = (C.splitmix64_np(np.arange(nw, dtype=np.uint64) + np.uint64(0x5DF5)) % np.uint64(len(words))).astype(np.int64)
    lens = wl[idx]
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
    total = int(lens.sum())
    within = np.arange(total) - np.repeat(starts, lens)
    flat = vocab[np.repeat(wo[idx], lens) + within][:base_n]
    reps = (nbytes + base_n - 1) // base_n
    return np.tile(flat, reps)[:nbytes]


def main():
    pending, hosts = [], {}
    eng = HipVariableSha256HashEngine()
    batch = DeviceBatch(eng, nbuf=NBUF, buf_len=L)
    for ds in SETS:
        if ds == "random":
            batch.fill_streams(first_stream=0, bufs_per_stream=256)
        elif ds == "mixed":  # every other buffer word salad: half the chunks compress, half do not
            batch.fill_streams(first_stream=0, bufs_per_stream=256)
            txt = torch.from_numpy(text_corpus((NBUF // 2) * L)).to(batch.data.device)
            batch.data.view(NBUF, L)[1::2].copy_(txt.view(NBUF // 2, L))
        else:
            batch.data.copy_(torch.from_numpy(text_corpus(NBUF * L)).to(batch.data.device))
        batch.run()
        torch.cuda.synchronize()
        recs = batch.record_table()
        n = recs.shape[0]
        for mname in MODES:
            mode = Z.MODES[mname]
            comp = HipLz4Compressor(mode)
            src_off, src_len, dst_off, total = comp.plan_records(recs, uniform_len=L)
            out = torch.empty(int(total.item()) + 16, dtype=torch.uint8, device="cuda")
            dst_len = torch.empty(n, dtype=torch.int32, device="cuda")
            s = torch.cuda.current_stream()
            # warm: >= 0.2 s of launches so the clocks are up after the CPU-baseline pauses
            tw = time.perf_counter()
            while time.perf_counter() - tw < 0.2:
                comp.compress_device(batch.data, src_off, src_len, out, dst_off, dst_len)
                torch.cuda.synchronize()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record(s)
            for _ in range(REPS):
                comp.compress_device(batch.data, src_off, src_len, out, dst_off, dst_len)
            ev[1].record(s)
            torch.cuda.synchronize()
            ms = ev[0].elapsed_time(ev[1]) / REPS
            nbytes = NBUF * L
            clen = int(dst_len.sum().item())
            # spot check against the oracle
            host = hosts.setdefault(ds, batch.data.cpu().numpy())
            so, sl, do, dl = (t.cpu().numpy() for t in (src_off, src_len, dst_off, dst_len))
            ob = out.cpu().numpy()
            rng = np.random.default_rng(1)
            for i in rng.integers(0, n, 32):
                chunk = host[int(so[i]): int(so[i]) + int(sl[i])]
                assert ob[int(do[i]): int(do[i]) + int(dl[i])].tobytes() == Z.compress_framed(chunk, mode), i
            # read side: decode the framed records back on the GPU (round trip checked)
            back = torch.empty(nbytes + 16, dtype=torch.uint8, device="cuda")
            blen = torch.empty(n, dtype=torch.int32, device="cuda")
            comp.decompress_device(out, dst_off, dst_len, back, src_off, src_len, blen)
            torch.cuda.synchronize()
            ev[0].record(s)
            for _ in range(REPS):
                comp.decompress_device(out, dst_off, dst_len, back, src_off, src_len, blen)
            ev[1].record(s)
            torch.cuda.synchronize()
            dms = ev[0].elapsed_time(ev[1]) / REPS
            assert torch.equal(blen, src_len) and torch.equal(back[:nbytes], batch.data[:nbytes])
            pending.append((ds, mname, mode, n, nbytes, ms, clen, so, sl, dms))
            comp.destroy()
    eng.destroy()
    # CPU oracle (C, THREADS pthreads) on a bounded sample of the same chunks -- after every GPU
    # measurement: a 16-thread CPU phase between two GPU timings halves the second one on the box
    for ds, mname, mode, n, nbytes, ms, clen, so, sl, dms in pending:
        host = hosts[ds]
        rng = np.random.default_rng(2)
        order = rng.permutation(n)
        k = min(n, 2048)
        while True:
            sel = np.sort(order[:k])
            _, cpu_secs = Z.compress_batch(host, so[sel], sl[sel], mode, THREADS)
            if cpu_secs >= CPU_SECS or k >= n:
                break
            k = min(n, int(k * max(2.0, CPU_SECS / max(cpu_secs, 1e-3))))
        done_bytes = int(sl[sel].sum())
        # the image's optimised liblz4 on the same sample (compress, then decode its own blocks)
        sys_leg = None
        if Z.system_lz4() is not None:
            s_off, s_len = so[sel], sl[sel]
            room = s_len + s_len // 255 + 16

            def timed(fn):
                tot, reps, r = 0.0, 0, None
                while reps == 0 or tot < max(0.5, CPU_SECS / 4):
                    r = fn()
                    tot += r[3]
                    reps += 1
                return r, tot / reps

            (cout, coffs, clens, _), ct = timed(lambda: Z.system_batch(False, host, s_off, s_len, room, THREADS))
            (_, _, dlens, _), dt = timed(lambda: Z.system_batch(True, cout, coffs, clens, s_len, THREADS))
            assert (dlens == s_len).all()
            sys_leg = {"compress_gibps": round(done_bytes / ct / 2**30, 3),
                       "decompress_gibps": round(done_bytes / dt / 2**30, 3), "threads": THREADS,
                       "sample_chunks": int(k),
                       "kind": "system liblz4 (LZ4_compress_default / LZ4_decompress_safe, V19 parse)"}
        print(json.dumps({
            "bench": "lz4_unique_chunks", "data": ds, "mode": mname, "chunks": int(n),
            "input_gib": round(nbytes / 2**30, 3), "kernel_ms": round(ms, 3),
            "gibps": round(nbytes / (ms / 1e3) / 2**30, 1), "ratio": round(nbytes / max(clen, 1), 3),
            "decompress_ms": round(dms, 3), "decompress_gibps": round(nbytes / (dms / 1e3) / 2**30, 1),
            "cpu_baseline": {"gibps": round(done_bytes / cpu_secs / 2**30, 3), "threads": THREADS,
                             "sample_chunks": int(k), "kind": "port (oracle/lz4_ref.c)"},
            "cpu_liblz4": sys_leg,
        }), flush=True)


if __name__ == "__main__":
    main()
