#!/usr/bin/env python3
"""AES-CBC of stored chunk records on one MI355X: device GiB/s.

Workload: NBUF write buffers of 256 KiB (default 4096 = 1 GiB) chunked by the engine with the
reference parameters; every chunk becomes an uncompressed putChunk record [int -1][chunk]
(HashBlobArchive.java:1281-1291) encrypted with AES-256/CBC/PKCS5 under one key and IV (the
prefix is framed on the fly, plen = 4).  Reports the encrypt kernel's device time (HIP events on
the launch stream, scheduling kernels included) per table-layout variant (SDFS_AES_VARIANT), the
decryption time of the same records, and the CPU oracle (oracle/aes_ref.c, byte-form FIPS-197,
no AES-NI) on a sample with THREADS host threads.  One JSON line per variant."""
import json
import os
import shutil
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import aes_oracle as A  # noqa: E402  (CPU baseline and spot checks only)
from sdfs_amd import HipVariableSha256HashEngine  # noqa: E402
from sdfs_amd.aes import HipEncryptUtils  # noqa: E402
from sdfs_amd.device import DeviceBatch  # noqa: E402

NBUF = int(os.environ.get("NBUF", "4096"))
REPS = int(os.environ.get("REPS", "5"))
THREADS = int(os.environ.get("THREADS", "16"))
CPU_SECS = float(os.environ.get("CPU_SECS", "6"))
VARIANTS = [int(v) for v in os.environ.get("VARIANTS", "7").split(",") if v]
UNIFORM = int(os.environ.get("UNIFORM", "0"))
L = 262144
KEY = A.key_from_passphrase("bench passphrase")
IV = bytes(range(16))


def openssl_speed(threads: int):
    """AES-256-CBC encrypt throughput of the host's openssl (AES-NI) on 8 KiB records, `threads`
    processes: the fastest CPU form of the same cipher on this box (GB/s), or None."""
    exe = shutil.which("openssl")
    if not exe:
        return None
    cmd = [exe, "speed", "-evp", "aes-256-cbc", "-bytes", "8192", "-seconds", "2"]
    if threads > 1:
        cmd[2:2] = ["-multi", str(threads)]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=60)
    except (subprocess.TimeoutExpired, OSError):
        return None
    for line in r.stdout.splitlines()[::-1]:
        parts = line.split()
        if parts and parts[-1].endswith("k") and (parts[0] in ("evp", "AES-256-CBC", "aes-256-cbc")):
            return round(float(parts[-1][:-1]) * 1e3 / 2**30, 2)
    return None


def main():
    eng = HipVariableSha256HashEngine()
    batch = DeviceBatch(eng, nbuf=NBUF, buf_len=L)
    batch.fill_streams(first_stream=0, bufs_per_stream=256)
    batch.run()
    torch.cuda.synchronize()
    recs = batch.record_table().cpu().numpy()
    n = recs.shape[0]
    meta = recs[:, 40:48].copy().view(np.uint32).reshape(n, 2)
    bid = recs[:, 32:40].copy().view(np.uint64).reshape(n)
    src_off = (bid.astype(np.int64) * L + meta[:, 0].astype(np.int64))
    src_len = meta[:, 1].astype(np.int64)
    if UNIFORM:  # probe: equal-length records (no long-record critical path)
        n = NBUF * L // UNIFORM
        src_off = np.arange(n, dtype=np.int64) * UNIFORM
        src_len = np.full(n, UNIFORM, np.int64)
    room = (src_len + 4) // 16 * 16 + 16
    dst_off = np.concatenate([[0], np.cumsum(room[:-1])]).astype(np.int64)
    dev = batch.data.device
    d_soff = torch.from_numpy(src_off).to(dev)
    d_slen = torch.from_numpy(src_len.astype(np.int32)).to(dev)
    d_doff = torch.from_numpy(dst_off).to(dev)
    out = torch.empty(int(room.sum()) + 16, dtype=torch.uint8, device=dev)
    dlen = torch.empty(n, dtype=torch.int32, device=dev)
    back = torch.empty_like(out)
    blen = torch.empty(n, dtype=torch.int32, device=dev)
    nbytes = int(src_len.sum())
    s = torch.cuda.current_stream()
    host = None
    for var in VARIANTS:
        os.environ["SDFS_AES_VARIANT"] = str(var)
        c = HipEncryptUtils(KEY)
        # warm: >= 0.2 s of launches so the clocks are up after the CPU-baseline pauses
        tw = time.perf_counter()
        while time.perf_counter() - tw < 0.2:
            c.encrypt_device(batch.data, d_soff, d_slen, out, d_doff, dlen, iv=IV, nz_prefix=-1)
            torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ev[0].record(s)
        for _ in range(REPS):
            c.encrypt_device(batch.data, d_soff, d_slen, out, d_doff, dlen, iv=IV, nz_prefix=-1)
        ev[1].record(s)
        ev[2].record(s)
        for _ in range(REPS):
            c.decrypt_device(out, d_doff, dlen, back, d_doff, blen, iv=IV)
        ev[3].record(s)
        torch.cuda.synchronize()
        enc_ms = ev[0].elapsed_time(ev[1]) / REPS
        dec_ms = ev[2].elapsed_time(ev[3]) / REPS
        # spot checks against the oracle and the round trip
        if host is None:
            host = batch.data.cpu().numpy()
        ob, dl, bl = out.cpu().numpy(), dlen.cpu().numpy(), blen.cpu().numpy()
        rng = np.random.default_rng(var)
        for i in rng.integers(0, n, 24):
            chunk = host[src_off[i]: src_off[i] + src_len[i]]
            want = A.cbc_encrypt(KEY, IV, chunk, prefix=b"\xff\xff\xff\xff")
            assert ob[dst_off[i]: dst_off[i] + dl[i]].tobytes() == want, i
        assert (bl == src_len + 4).all()
        res = {"bench": "aes256_cbc_records", "variant": var, "uniform_len": UNIFORM or None, "records": int(n), "input_gib": round(nbytes / 2**30, 3),
               "mean_record_bytes": round(nbytes / n + 4, 1), "encrypt_ms": round(enc_ms, 3),
               "encrypt_gibps": round(nbytes / (enc_ms / 1e3) / 2**30, 1), "decrypt_ms": round(dec_ms, 3),
               "decrypt_gibps": round(nbytes / (dec_ms / 1e3) / 2**30, 1)}
        print(json.dumps(res), flush=True)
        c.destroy()
    eng.destroy()
    # CPU baselines after every GPU measurement (a 16-thread CPU phase between two GPU timings
    # slows the second one down on the box)
    rng = np.random.default_rng(0)
    order = rng.permutation(n)
    k = min(n, 256)
    while True:
        sel = np.sort(order[:k])
        _, cpu_secs = A.cbc_encrypt_batch(KEY, IV, host, src_off[sel].astype(np.uint64), src_len[sel],
                                          prefix=b"\xff\xff\xff\xff", nthreads=THREADS)
        if cpu_secs >= CPU_SECS or k >= n:
            break
        k = min(n, int(k * max(2.0, CPU_SECS / max(cpu_secs, 1e-3))))
    print(json.dumps({"bench": "aes256_cbc_records_cpu",
                      "cpu_baseline": {"gibps": round(int(src_len[sel].sum()) / cpu_secs / 2**30, 4),
                                       "threads": THREADS, "sample_records": int(k),
                                       "kind": "port (oracle/aes_ref.c, byte-form FIPS-197)"},
                      "cpu_openssl_aesni": {"gibps_1thread": openssl_speed(1), "gibps": openssl_speed(THREADS),
                                            "threads": THREADS, "kind": "openssl speed -evp aes-256-cbc, 8 KiB"}}),
          flush=True)


if __name__ == "__main__":
    main()
