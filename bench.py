#!/usr/bin/env python3
"""bench.py — device-resident GiB/s of variable-block CDC + fingerprint (BASELINE.json metric).

Workload (BASELINE.json configs[1]): per GPU, 64 independent synthetic write
streams x 64 MiB, cut into CHUNK_LENGTH = 256 KiB write buffers (16384 buffers, 4 GiB) resident in
HBM before the timed region; every buffer is chunked from a fresh CDC state.  The headline uses
the metric's chunk mix, a 4 KiB mean: min-variable-segment-size = 2 (minLen 2047,
Config.java:145-148) and an 11-bit boundary predicate, with the reference's other parameters
(P = 0x26CE86126EF863, W = 48, maxLen 32768, SHA-256); the reference-default mix (minLen 4095,
12-bit predicate, ~8 KiB mean) is reported beside it (`at_ref_default`).
One step = scan + cut resolution + SHA-256 of every chunk of the 4 GiB; at N > 1 the step also
all-gathers the fingerprint table (48-byte records) over RCCL.  Weak scaling: GPU r owns streams
[64r, 64r+64).

N > 1 runs two ways, the same work either way:
* under a launcher (torch.distributed.run, the driver's form): one process per GPU, WORLD_SIZE
  must equal --gpus, the exchange over torch.distributed "nccl" (RCCL; sdfs_amd/dist.py);
* without one: ONE process drives all N GPUs through one engine whose device set is GPUs 0..N-1
  (include/sdfs_cdc.h "Devices"), and the engine all-gathers the tables itself over RCCL
  (sdfs_cdc_allgather_records, pipelined one step behind production).

Production device path: one engine, steps alternating between two HIP streams (the engine's
workspace ring keeps two batches in flight, so one batch's scan fills the tail of the other's
fingerprinting).  The one-stream rate is reported beside it (`one_stream`).

Prints ONE JSON line on rank 0 (contract in the task statement); diagnostics go to stderr.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md); 6.29 TB/s measured float4 copy
# The fingerprint kernel is bound by VALU issue, not by HBM: its SHA-256 compression runs at the
# issue rate of its own instruction mix (scripts/valu_issue_mb.hip, profiles/r05/valu_issue/: real
# cycles per wave64 instruction per SIMD, 2.4 for xor/add/shift, ~2.5 bitop3, ~4.2 alignbit/add3/perm,
# 3.9 for the compression's mix at 4 waves per SIMD; no order, register assignment or ILP form of the
# round beats it).  The ceiling is measured live (sha_ceiling below) and the roofline reports the
# kernel's compressed bytes per second against it next to the HBM fraction.
PROBE_LIB = os.path.join(ROOT, "tools", "libsdfs_probe.so")
METRIC = "device-resident GiB/s CDC+fingerprint, 4 KiB-mean chunks, 1/2/4/8 MI355X"


def sha_ceiling(local: int, waves_per_simd: int = 4) -> float:
    """GB/s of 64-byte blocks the production sha256_compress reaches register-only on every CU of
    this GPU, now, at chunk_hash's occupancy (4 waves per SIMD: 120 VGPRs): the VALU issue ceiling
    of the fingerprint (tools/probe_kernels.hip, a measurement library beside the product)."""
    import ctypes

    lib = ctypes.CDLL(PROBE_LIB)
    f = lib.sdfs_probe_sha256_ceiling
    f.argtypes = [ctypes.c_int] * 4 + [ctypes.POINTER(ctypes.c_double)] * 2
    g, ms = ctypes.c_double(), ctypes.c_double()
    # 2000 blocks per lane (~5 ms per launch): the launch's own ramp and drain stay well under 1 %
    # (200 blocks made the ceiling ~3 % low: the fingerprint then appeared to beat it at 3 waves/SIMD)
    rc = f(local, waves_per_simd, 2000, 3, ctypes.byref(g), ctypes.byref(ms))
    if rc:
        raise RuntimeError(f"sdfs_probe_sha256_ceiling failed: {rc}")
    return g.value


_probe = None


def probe_lib():
    import ctypes

    global _probe
    if _probe is None:
        _probe = ctypes.CDLL(PROBE_LIB)
        _probe.sdfs_probe_exchange_proxy_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                            ctypes.c_int, ctypes.c_double, ctypes.c_void_p]
    return _probe


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def roofline_block(nbytes: int, hash_ms: float, ms_step: float, sha_blocks: int, ceiling: float,
                   traffic, traffic_src, kernel_ms_source: str, hash_ms_live=None) -> dict:
    """The bench line's roofline for the dominant kernel (chunk_hash).  The top level is the
    contract's HBM roofline: algorithmic bytes per launch (the input it fingerprints) over its
    one-stream launch duration, against the 8 TB/s HBM peak.  The kernel's real limiter is VALU
    issue of the SHA-256 mix; `valu` reports its compressed bytes against the live issue ceiling."""
    t_dom = hash_ms / 1e3
    achieved = nbytes / t_dom / 1e9 if t_dom > 0 else 0.0
    valu_gbps = sha_blocks * 64 / t_dom / 1e9 if t_dom > 0 else 0.0
    return {
        "bound": "hbm",
        "limiter": "valu",
        "kernel": "chunk_hash",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBPS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBPS, 4),
        "traffic": traffic,
        "traffic_source": traffic_src,
        "kernel_ms": round(hash_ms, 4),
        "kernel_ms_source": kernel_ms_source,
        "algorithmic_bytes_per_launch": nbytes,
        "two_stream_launch_ms": round(hash_ms_live, 4) if hash_ms_live else None,
        "achieved_per_step": round(nbytes / (ms_step / 1e3) / 1e9, 1),
        "frac_per_step": round(nbytes / (ms_step / 1e3) / 1e9 / HBM_PEAK_GBPS, 4),
        "valu": {
            "ceiling_gbps": round(ceiling, 1),
            "achieved_gbps": round(valu_gbps, 1),
            "frac": round(valu_gbps / ceiling, 4) if ceiling > 0 else None,
            "unit": "GB/s of 64-byte SHA-256 blocks (chunk bytes + padding blocks)",
            "sha_blocks_per_launch": sha_blocks,
            "ceiling_source": ("production sha256_compress, register-resident data, every CU at 4 waves/SIMD, "
                               "timed in this process (tools/probe_kernels.hip)"),
            "note": ("the kernel is bound by VALU issue of its SHA-256 instruction mix, not by HBM: the top-level "
                     "frac is of the 8 TB/s HBM peak, this one of the measured issue ceiling"),
        },
    }


def sha_blocks_of(torch, batch) -> int:
    """What chunk_hash compresses per launch: every chunk's 64-byte blocks incl. its padding block(s)."""
    valid = torch.arange(batch.cap, device=batch.lens.device)[None, :] < batch.counts[:, None]
    lens = batch.lens.view(batch.nbuf, batch.cap).to(torch.int64)
    return int((((lens + 8) // 64 + 1) * valid).sum().item())


def table_digest(torch, rows) -> str:
    """SHA-256 of a record table's bytes (compares the exchanged table across bench forms)."""
    import hashlib

    return hashlib.sha256(rows.contiguous().cpu().numpy().tobytes()).hexdigest()


def exchange_check(torch, dist, gathered, counts, own_slot, total, rank, world, device) -> dict:
    """Self-check of one exchanged step (collective: every rank calls it): every rank's count equals
    its batch's chunk total, and this rank's rows of the gathered table (rank r's rows at
    [r * max, r * max + counts[r])) are the records its engine wrote into its slot."""
    mx = max(counts)
    mine = gathered[rank * mx: rank * mx + counts[rank]]
    tot = torch.tensor([total], device=device, dtype=torch.int64)
    tots = [torch.zeros_like(tot) for _ in range(world)]
    dist.all_gather(tots, tot)
    tots = [int(x.item()) for x in tots]
    return {"counts": list(counts), "stride": mx, "counts_match": list(counts) == tots,
            "rows_match": bool(torch.equal(mine, own_slot[: counts[rank]])),
            "table_sha256": [table_digest(torch, mine)] if rank == 0 else None}


def cpu_baseline_block(args, cfg):
    aff = len(os.sched_getaffinity(0))
    quota = cpu_quota()
    th = args.cpu_threads or max(1, min(16 if quota is None else int(quota), aff))
    p_kw = dict(min_len=cfg.min_len, pred_mask=cfg.pred_mask)
    log(f"cpu baseline: {th} threads, ~{args.cpu_secs}s sample")
    cpu = cpu_baseline(args.cpu_secs, th, p_kw)
    if th > 1 and args.cpu_1t_secs > 0:  # T = all cores and T = 1
        one = cpu_baseline(args.cpu_1t_secs, 1, p_kw)
        cpu["one_thread"] = {"value": one["value"], "sample": one["sample"]}
    cpu["cpu_model"] = cpu_model()
    cpu["affinity_cpus"] = aff
    cpu["cpu_quota"] = quota
    return cpu


def cpu_baseline(target_secs: float, threads: int, p_kw: dict):
    """The CPU restatement of the path (oracle/cdc_fast.c: table-driven Rabin loop + OpenSSL
    EVP SHA-256, i.e. SHA-NI on this host as HotSpot's intrinsic would use) on a bounded sample of
    the same synthetic workload, timed on this host's cores: a reported baseline, not the target."""
    from oracle import cdc_oracle as O

    p = O.Params(**p_kw)
    t_cal, _, by = O.bench_fast(p, threads * 2, 262144, threads)
    rate = by / max(t_cal, 1e-6)
    nbuf = max(threads * 4, int(rate * target_secs / 262144) // threads * threads)
    secs, chunks, nbytes = O.bench_fast(p, nbuf, 262144, threads, buffers_per_stream=256)
    return dict(value=round(nbytes / secs / 2**30, 4), unit="GiB/s", cores=threads, kind="port",
                sample=f"{nbuf} x 256 KiB synthetic write buffers (streams 0..{(nbuf - 1) // 256}, "
                       f"same generator/params), {threads} threads, {secs:.1f} s, "
                       f"{nbytes / max(chunks, 1):.0f} B mean chunk; table-driven Rabin + OpenSSL SHA-256 "
                       f"(CPU restatement, not the Java reference)")


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def load_traffic(name: str, params: str):
    """HBM bytes per launch of `name` from the committed PMC passes (profiles/pmc_traffic.json),
    only when they were measured on this exact configuration; with the source label."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))
    except Exception:
        return None, None
    d = d.get("by_params", {}).get(params) or (d if d.get("params") == params else None)
    if not d or name not in d:
        return None, None
    return d[name].get("hbm_bytes_per_launch"), f"{d.get('source', '?')} (commit {d.get('commit', '?')})"


def cpu_quota():
    """The cgroup CPU quota (cpu.max) in CPUs, or None when there is none (on the GPU box nproc and
    the affinity mask show the whole machine; a job's share is 16 CPUs per GPU)."""
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return round(int(q) / int(period), 2)
    except Exception:
        pass
    return None


def git_head() -> str:
    """HEAD of the tree, or (on the GPU box, which gets no .git) the commit `make` recorded."""
    try:
        h = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"], capture_output=True,
                           text=True, timeout=10).stdout.strip()
        if h:
            return h
    except Exception:
        pass
    try:
        return "built from " + open(os.path.join(ROOT, "sdfs_amd", "BUILD_COMMIT")).read().strip()
    except OSError:
        return "unknown"


class StreamRunner:
    """Steps rotate over `depth` HIP streams on ONE engine (2 by default), each with its own output
    set (DeviceBatch) over the same resident input: `depth` batches in flight (the engine's
    workspace ring holds three)."""

    def __init__(self, torch, eng, batch, cs, DeviceBatch, nbuf, buf_len, device, depth=2):
        self.torch = torch
        self.batches = [batch] + [DeviceBatch(eng, nbuf=nbuf, buf_len=buf_len, device=device)
                                  for _ in range(depth - 1)]
        for b in self.batches[1:]:
            b.data = batch.data
        self.streams = [cs] + [torch.cuda.Stream(device=device) for _ in range(depth - 1)]
        self.k = 0

    def step(self, buffer_id_base, exchange=None):
        i = self.k % len(self.batches)
        self.k += 1
        b, s = self.batches[i], self.streams[i]
        rec = None
        if exchange is not None and exchange.direct:
            rec = exchange.acquire(stream=s)  # the engine writes its records into the exchange slot
            b.set_records(rec)
        b.run(buffer_id_base=buffer_id_base, stream=s.cuda_stream)
        if exchange is not None:
            exchange.submit(rec if rec is not None else b.recs.view(-1, 48), b.total, stream=s)

    def identical(self) -> bool:
        t = self.torch
        t.cuda.synchronize()
        a = self.batches[0]
        return all(bool(t.equal(a.record_table(), b.record_table()) and t.equal(a.counts, b.counts))
                   for b in self.batches[1:])


def timed(torch, dist, world, fn, steps):
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    return el


def threads_sweep(eng_cfg, device, host, buf_len, thread_counts, mode="fill"):
    """SDFS's own calling pattern: T C threads, each calling getChunks on one 256 KiB buffer at a
    time through the C-ABI (coalesced into shared GPU passes); rate and per-call latency.  mode
    "fill" is the JNI glue's entry point (sdfs_cdc_get_chunks_fill: the byte[] copied once,
    straight into the engine's pinned staging)."""
    from sdfs_amd import HashFunctionPool
    from tools import threads as T

    out = {"entry": "sdfs_cdc_get_chunks_fill (JNI glue)" if mode == "fill" else "sdfs_cdc_get_chunks"}
    eng = HashFunctionPool(eng_cfg, device=device).getHashEngine()
    # warm at the highest concurrency of the sweep, so every slot and lane has carried a pass
    tmax = max(thread_counts) if thread_counts else 8
    T.getchunks(eng, tmax, host, buf_len, max(256, 4 * tmax), mode=mode)
    start = eng.queue_stats()
    for th in thread_counts:
        calls = max(512, th * 48)  # >= 48 calls per thread: a few ms per point is too noisy to compare
        r, _ = T.getchunks(eng, th, host, buf_len, calls, mode=mode)
        b0 = eng.queue_stats()
        out[str(th)] = {"gibps": round(r.gibps, 3), "p50_us": round(r.p50_us, 1), "p99_us": round(r.p99_us, 1),
                        "mean_us": round(r.mean_us, 1), "calls": r.calls, "errors": r.first_error}
        out[str(th)]["_stats"] = b0
    # batches per sweep point from the cumulative queue statistics
    prev = start
    for th in thread_counts:
        cur = out[str(th)].pop("_stats")
        nb, nr = cur[0] - prev[0], cur[1] - prev[1]
        out[str(th)]["calls_per_gpu_pass"] = round(nr / max(nb, 1), 1)
        prev = cur
    eng.destroy()
    return out

def main_device_set(args):
    """--gpus N > 1 without a launcher: ONE process, one engine whose device set is GPUs 0..N-1.
    GPU d owns streams [64d, 64d+64) (weak scaling, as one rank per GPU would), each GPU keeps two
    batches in flight on two streams, and the engine all-gathers the record tables in process over
    RCCL one step behind production (sdfs_amd/dist.py DeviceSetExchange)."""
    import torch

    from sdfs_amd import HipVariableSha256HashEngine, SdfsConfig
    from sdfs_amd.device import DeviceBatch
    from sdfs_amd.dist import DeviceSetExchange, shard_streams

    n = args.gpus
    if torch.cuda.device_count() < n:
        log(f"bench.py: --gpus {n} but only {torch.cuda.device_count()} GPUs are visible")
        sys.exit(2)
    cfg = SdfsConfig(chunk_length=args.buf_kib * 1024, min_len=args.min_seg_kib * 1024 - 1,
                     pred_mask=(1 << args.mask_bits) - 1, hash_type=args.hash_type)
    eng = HipVariableSha256HashEngine(config=cfg, device=-1, device_mask=(1 << n) - 1)
    assert eng.device_ordinals() == list(range(n))
    buf_len = args.buf_kib * 1024
    bufs_per_stream = args.stream_mib * 1024 // args.buf_kib
    batches, streams = [], []
    for d in range(n):
        dev = f"cuda:{d}"
        with torch.cuda.device(d):
            sh = shard_streams(args.streams * n, n, d)
            nbuf = len(sh) * bufs_per_stream
            b0 = DeviceBatch(eng, nbuf=nbuf, buf_len=buf_len, device=dev)
            b0.fill_streams(first_stream=sh.start, bufs_per_stream=bufs_per_stream)
            b1 = DeviceBatch(eng, nbuf=nbuf, buf_len=buf_len, device=dev)
            b1.data = b0.data
            batches.append([b0, b1])
            streams.append([torch.cuda.Stream(device=d), torch.cuda.Stream(device=d)])
    for d in range(n):
        torch.cuda.synchronize(d)
    nbytes = batches[0][0].nbytes
    cap_rec = batches[0][0].nbuf * batches[0][0].cap
    ex = DeviceSetExchange(eng, cap_rec, [f"cuda:{d}" for d in range(n)])

    def step(i):
        for d in range(n):
            b, s = batches[d][i % 2], streams[d][i % 2]
            b.set_records(ex.acquire(i, d, s))
            b.run(buffer_id_base=d * b.nbuf, stream=s.cuda_stream)
            ex.produced(i, d, b.total, s)
        if i >= 1:
            ex.exchange(i - 1)

    def sync_all():
        for d in range(n):
            torch.cuda.synchronize(d)

    t_ramp = time.perf_counter()
    i = 0
    while time.perf_counter() - t_ramp < args.ramp_secs:
        step(i)
        i += 1
    for _ in range(args.warmup):
        step(i)
        i += 1
    if i:
        ex.exchange(i - 1)
    sync_all()
    eng.set_timing_stages(args.steps, ("chunk_hash",))
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(i + k)
    last = i + args.steps - 1
    ex.exchange(last)
    sync_all()
    elapsed = time.perf_counter() - t0
    hash_ms_live = [eng.kernel_times(d).get("chunk_hash", 0.0) for d in range(n)]
    eng.set_timing(0)
    value = n * nbytes * args.steps / elapsed / 2**30
    ms_step = elapsed / args.steps * 1e3

    # the exchanged table of the last timed step, checked: every device's count is its batch's
    # total, and device j's rows in GPU 0's gathered table are device j's own records
    counts, stride = ex.results[-1]
    k_last = last % ex.nslots
    totals = [int(batches[d][last % 2].total.item()) for d in range(n)]
    g0 = ex.gathered[0][last % 2]
    rows_match = all(
        torch.equal(g0[j * stride: j * stride + counts[j]].cpu(), ex.slots[j][k_last][: counts[j]].cpu())
        for j in range(n))
    table_sha = [table_digest(torch, ex.slots[j][k_last][: counts[j]]) for j in range(n)]

    # The roofline's launch duration, per GPU: chunk_hash timed with HIP events over a one-stream
    # region (stream-ordered, so nothing overlaps the kernel; the two-stream region's launches are
    # stretched by the other batch's scan and are reported beside it only)
    def one_all():
        for d in range(n):
            batches[d][0].run(buffer_id_base=d * batches[d][0].nbuf, stream=streams[d][0].cuda_stream)

    for _ in range(2):
        one_all()
    sync_all()
    eng.set_timing_stages(args.steps, ("chunk_hash",))
    t1 = time.perf_counter()
    for _ in range(args.steps):
        one_all()
    sync_all()
    el_one = time.perf_counter() - t1
    hash_ms = [eng.kernel_times(d).get("chunk_hash", 0.0) for d in range(n)]
    eng.set_timing(0)
    with torch.cuda.device(0):
        ceiling = sha_ceiling(0)  # right after the one-stream region: the same clock regime
        sha_blocks = sha_blocks_of(torch, batches[0][0])
    params = (f"P=0x26CE86126EF863 W=48 minLen={cfg.min_len} maxLen={cfg.max_len} "
              f"pred=(fp&{cfg.pred_mask:#x})==0 n>minLen {args.hash_type}")
    traffic, traffic_src = load_traffic("chunk_hash", params)
    roof = roofline_block(nbytes, hash_ms[0], ms_step, sha_blocks, ceiling, traffic, traffic_src,
                          "HIP events around chunk_hash on GPU 0's launch stream over a one-stream region of "
                          f"{args.steps} steps per GPU (stream-ordered: nothing overlaps the kernel)",
                          hash_ms_live[0])
    cpu = cpu_baseline_block(args, cfg) if args.cpu_secs > 0 else None
    res = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": n,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (counter-based SplitMix64 streams, 0% duplicate), resident in HBM",
        "config": {
            "workload": f"{args.streams} streams x {args.stream_mib} MiB per GPU, CHUNK_LENGTH {buf_len} B "
                        f"({batches[0][0].nbuf} buffers, {nbytes / 2**30:.2f} GiB per GPU), fresh CDC state per buffer",
            "params": params,
            "mean_chunk_bytes": round(n * nbytes / max(sum(totals), 1), 1),
            "chunks_per_gpu_step": totals,
            "streams_in_flight": 2,
            "exchange": "in-process RCCL all-gather of the 48-B fingerprint records by the engine "
                        "(sdfs_cdc_allgather_records), pipelined one step behind production",
            "exchange_last_step": {"counts": counts, "stride": stride, "counts_match": counts == totals,
                                   "rows_match": rows_match, "table_sha256": table_sha},
            "parallelism": f"device set of {n} GPUs in one process (streams sharded per GPU)",
        },
        "kernels_ms": {"chunk_hash_per_gpu": [round(x, 4) for x in hash_ms],
                       "chunk_hash_two_stream_per_gpu": [round(x, 4) for x in hash_ms_live]},
        "one_stream": {"streams_in_flight": 1, "value": round(n * nbytes * args.steps / el_one / 2**30, 3),
                       "ms_per_step": round(el_one / args.steps * 1e3, 4)},
        "roofline": roof,
        "records_sha256": table_digest(torch, batches[0][0].record_table()),
        "cpu_baseline": cpu,
        "commit": git_head(),
    }
    print(json.dumps(res), flush=True)
    eng.destroy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--streams", type=int, default=64, help="write streams per GPU")
    ap.add_argument("--stream-mib", type=int, default=64)
    ap.add_argument("--buf-kib", type=int, default=256, help="CHUNK_LENGTH in KiB")
    ap.add_argument("--cpu-secs", type=float, default=12.0, help="CPU baseline sample size (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--cpu-1t-secs", type=float, default=3.0, help="single-thread CPU baseline sample (0 = skip)")
    ap.add_argument("--e2e-mib", type=int, default=1024, help="host->GPU->host batch measurement size (0 = skip)")
    ap.add_argument("--threads", default="auto",
                    help="getChunks caller-thread counts for the coalescing-queue sweep ('' = skip; auto = "
                         "1,8,32,3 x the CPU quota (SDFS's default write-threads, Main.java:211-212),64,128,256)")
    ap.add_argument("--threads-mode", default="fill", choices=["fill", "copy"],
                    help="fill: the JNI glue's entry point (the byte[] copied once, into pinned staging)")
    ap.add_argument("--min-seg-kib", type=int, default=2,
                    help="min-variable-segment-size (minLen = KiB*1024-1; 2 = the metric's 4 KiB-mean mix, "
                         "4 = the reference default)")
    ap.add_argument("--mask-bits", type=int, default=11,
                    help="boundary predicate (fp & (2^bits-1)) == 0 (11 = the 4 KiB-mean mix, 12 = the default "
                         "knob, SURVEY.md A.3)")
    ap.add_argument("--other-mix", type=int, default=1,
                    help="also time the other mix (the reference default beside the 4 KiB mean, or vice versa)")
    ap.add_argument("--hash-type", default="VARIABLE_SHA256",
                    choices=["VARIABLE_SHA256", "VARIABLE_SHA256_160", "VARIABLE_MD5"])
    ap.add_argument("--ramp-secs", type=float, default=0.3, help="untimed clock ramp before the warmup steps")
    ap.add_argument("--streams-in-flight", type=int, default=2, choices=[1, 2, 3],
                    help="HIP streams the steps alternate on (2 = production: two batches in flight)")
    ap.add_argument("--compare", type=int, default=1, help="also time the other streams-in-flight mode (N = 1)")
    ap.add_argument("--exchange", type=int, default=-1,
                    help="record all-gather: -1 = when N > 1, 1 = also at N = 1 (exercises the path)")
    ap.add_argument("--inproc", type=int, default=0,
                    help="1: drive the GPUs from ONE process through a device-set engine even at N = 1 "
                         "(the default for N > 1 without a launcher)")
    ap.add_argument("--exchange-mode", default="direct", choices=["direct", "copy"],
                    help="direct: the engine writes records into the exchange slot; copy: snapshot copy")
    ap.add_argument("--exchange-proxy", type=int, default=0,
                    help="W > 1 (N = 1 only): project the W-rank exchange onto one GPU -- each step, a paced copy of "
                         "(W-1) x this GPU's record bytes on a side stream with RCCL's footprint (--proxy-wgs "
                         "workgroups for as long as xGMI at --proxy-gbps takes; tools/probe_kernels.hip)")
    ap.add_argument("--proxy-wgs", type=int, default=32, help="workgroups of the exchange proxy (RCCL channels)")
    ap.add_argument("--proxy-gbps", type=float, default=300.0, help="assumed per-GPU all-gather receive rate")
    ap.add_argument("--proxy-record-bytes", type=int, default=48, help="bytes per exchanged record")
    ap.add_argument("--proxy-prio", type=int, default=0, help="1: the proxy's stream at high priority")
    args = ap.parse_args()

    launched = "WORLD_SIZE" in os.environ
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if launched and world != args.gpus:
        log(f"bench.py: --gpus {args.gpus} but the launcher started {world} ranks (WORLD_SIZE); they must agree")
        sys.exit(2)
    if not launched and (args.gpus > 1 or args.inproc):
        return main_device_set(args)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(local)
    device = f"cuda:{local}"
    use_ex = world > 1 if args.exchange < 0 else bool(args.exchange)
    if use_ex or world > 1:
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        from sdfs_amd.dist import exchange_pg_options
        dist.init_process_group("nccl", device_id=torch.device(device), pg_options=exchange_pg_options())

    from sdfs_amd import HashFunctionPool, SdfsConfig
    from sdfs_amd.device import DeviceBatch
    from sdfs_amd.dist import RecordExchange, shard_streams

    cfg = SdfsConfig(chunk_length=args.buf_kib * 1024, min_len=args.min_seg_kib * 1024 - 1,
                     pred_mask=(1 << args.mask_bits) - 1, hash_type=args.hash_type)
    eng = HashFunctionPool(cfg, device=local).getHashEngine()
    buf_len = args.buf_kib * 1024
    bufs_per_stream = args.stream_mib * 1024 // args.buf_kib
    streams = shard_streams(args.streams * world, world, rank)
    nbuf = len(streams) * bufs_per_stream
    nbytes = nbuf * buf_len
    batch = DeviceBatch(eng, nbuf=nbuf, buf_len=buf_len, device=device)
    batch.fill_streams(first_stream=streams.start, bufs_per_stream=bufs_per_stream)
    torch.cuda.synchronize()
    cs = torch.cuda.current_stream()
    base_id = rank * nbuf
    nsf = args.streams_in_flight
    runner = StreamRunner(torch, eng, batch, cs, DeviceBatch, nbuf, buf_len, device, depth=max(nsf, 2))
    # N > 1: the one real exchange (all-gather of the fingerprint records), pipelined on a side
    # stream so step i's table travels while step i+1 is chunked (sdfs_amd/dist.py)
    ex = None
    if use_ex:
        direct = args.exchange_mode == "direct"
        # direct: a third slot, so a step's slot was all-gathered a step before it is rewritten
        ex = RecordExchange(batch.recs.view(-1, 48).shape[0], device, depth=2, slots=3 if direct else 2)
        ex.direct = direct

    proxy = None  # set after the warmup (--exchange-proxy): [side stream, dst, src, bytes]

    def proxy_after(stream):
        """The projected exchange of the step just issued on `stream`: the paced copy on a side
        stream behind the step's production, as RecordExchange runs RCCL behind it."""
        px, dst, src, nb = proxy
        ev = torch.cuda.Event()
        ev.record(stream)
        px.wait_event(ev)
        rc = probe_lib().sdfs_probe_exchange_proxy_launch(dst.data_ptr(), src.data_ptr(), nb, args.proxy_wgs,
                                                          ctypes.c_double(args.proxy_gbps), px.cuda_stream)
        if rc:
            raise RuntimeError(f"exchange proxy launch failed: {rc}")

    def step():
        if nsf >= 2:
            runner.step(base_id, ex)
            if proxy is not None:
                proxy_after(runner.streams[(runner.k - 1) % len(runner.streams)])
        else:
            rec = None
            if ex is not None and ex.direct:
                rec = ex.acquire(stream=cs)
                batch.set_records(rec)
            batch.run(buffer_id_base=base_id, stream=cs.cuda_stream)
            if ex is not None:
                ex.submit(rec if rec is not None else batch.recs.view(-1, 48), batch.total, stream=cs)
            if proxy is not None:
                proxy_after(cs)

    last_exchange = []

    def drain():
        if ex is not None:
            r = ex.flush()
            if r:
                last_exchange[:] = [r[-1], (ex.n - 1) % ex.nslots]

    # clock ramp: ~0.3 s of chunking before the W warmup steps (the GPU idles while the host sets
    # up and its clocks drop; a few 4.5 ms steps do not bring them back), outside the timed region
    t_ramp = time.perf_counter()
    while time.perf_counter() - t_ramp < args.ramp_secs:
        batch.run(buffer_id_base=base_id, stream=cs.cuda_stream)
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()
    drain()
    proxy_info = None
    if args.exchange_proxy > 1:
        if world != 1:
            raise SystemExit("--exchange-proxy projects N ranks onto one GPU: run it at N = 1")
        torch.cuda.synchronize()
        recs = int(batch.total.item())
        nb = ((args.exchange_proxy - 1) * recs * args.proxy_record_bytes + 15) // 16 * 16
        proxy = [torch.cuda.Stream(device=device, priority=-1 if args.proxy_prio else 0),
                 torch.empty(nb, dtype=torch.uint8, device=device),
                 torch.zeros(nb, dtype=torch.uint8, device=device), nb]
        # the proxy alone on the idle GPU (second launch: warm): its own duration, i.e. the
        # projected xGMI time when the copy keeps its pace
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        proxy_after(proxy[0])
        e0.record(proxy[0])
        proxy_after(proxy[0])
        e1.record(proxy[0])
        e1.synchronize()
        proxy_info = {"ranks": args.exchange_proxy, "bytes_per_step": nb, "records_per_gpu_step": recs,
                      "record_bytes": args.proxy_record_bytes, "workgroups": args.proxy_wgs,
                      "gbps": args.proxy_gbps, "high_priority": bool(args.proxy_prio),
                      "alone_ms": round(e0.elapsed_time(e1), 4)}
        for _ in range(2):
            step()
        torch.cuda.synchronize()
    # timed region: HIP events only around the dominant kernel (the roofline's launch duration)
    eng.set_timing_stages(args.steps, ("chunk_hash",))

    def timed_steps():
        for _ in range(args.steps):
            step()
        drain()

    elapsed = timed(torch, dist, world, timed_steps, 1)
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    hash_ms_live = eng.kernel_times().get("chunk_hash", 0.0)
    identical = runner.identical() if nsf >= 2 else None

    # per-stage breakdown (untimed, one stream, events around every kernel)
    nbd = max(3, min(args.steps, 10))
    eng.set_timing(nbd)
    for _ in range(nbd):
        batch.run(buffer_id_base=base_id, stream=cs.cuda_stream)
    torch.cuda.synchronize()
    kt = eng.kernel_times()
    eng.set_timing(0)
    counts, _, _, _, total = batch.host_results()
    sha_blocks = sha_blocks_of(torch, batch)
    records_sha = table_digest(torch, batch.record_table())
    # the exchanged table of the last timed step, checked: every rank's count, and this rank's rows
    # of the gathered table equal the records its engine wrote
    ex_check = None
    if ex is not None and last_exchange:
        (gathered, cl), k_last = last_exchange
        ex_check = exchange_check(torch, dist, gathered, cl, ex.slots[k_last], total, rank, world, device)

    # The roofline's launch duration: chunk_hash timed with HIP events over a one-stream timed
    # region (every step stream-ordered, so no other kernel shares the GPU with chunk_hash and its
    # launch duration is its own time).  With two batches in flight the headline region's launches
    # overlap the other batch's scan and are stretched beyond a step (reported beside it as
    # `two_stream_launch_ms`, not used for the roofline).  At N = 1 this region is also the other
    # in-flight mode's rate (`one_stream`).
    def one():
        batch.run(buffer_id_base=base_id, stream=cs.cuda_stream)

    other = None
    if nsf >= 2:
        for _ in range(2):
            one()
        eng.set_timing_stages(args.steps, ("chunk_hash",))
        el = timed(torch, dist, 1, one, args.steps)
        hash_ms_one = eng.kernel_times().get("chunk_hash", 0.0)
        eng.set_timing(0)
        other = {"streams_in_flight": 1, "value": round(nbytes * args.steps / el / 2**30, 3),
                 "ms_per_step": round(el / args.steps * 1e3, 4), "chunk_hash_ms": round(hash_ms_one, 4)}
    else:
        hash_ms_one = hash_ms_live
        if world == 1 and args.compare:
            def two():
                runner.step(base_id)

            for _ in range(2):
                two()
            el = timed(torch, dist, 1, two, args.steps)
            other = {"streams_in_flight": 2, "value": round(nbytes * args.steps / el / 2**30, 3),
                     "ms_per_step": round(el / args.steps * 1e3, 4)}
    if world > 1:
        other = None
        # every rank's one-stream chunk_hash launch (the roofline uses rank 0's)
        t = torch.tensor([hash_ms_one], device=device, dtype=torch.float64)
        per = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(per, t)
        hash_ms_ranks = [round(float(x.item()), 4) for x in per]
    else:
        hash_ms_ranks = [round(hash_ms_one, 4)]
    ceiling = sha_ceiling(local)  # right after the one-stream region: the same clock regime

    # the other chunk mix beside the headline: the reference default (minLen 4095, 12-bit) when
    # the headline is the metric's 4 KiB-mean mix (minLen 2047, 11-bit), and vice versa
    other_mix = None
    main_is_4k = (cfg.min_len, cfg.pred_mask) == (2047, 0x7FF)
    if world == 1 and args.other_mix:
        om_min, om_mask = (4095, 0xFFF) if main_is_4k else (2047, 0x7FF)
        cfg4 = SdfsConfig(chunk_length=buf_len, min_len=om_min, pred_mask=om_mask, hash_type=args.hash_type)
        e4 = HashFunctionPool(cfg4, device=local).getHashEngine()
        b4 = DeviceBatch(e4, nbuf=nbuf, buf_len=buf_len, device=device)
        b4.data = batch.data
        r4 = StreamRunner(torch, e4, b4, cs, DeviceBatch, nbuf, buf_len, device)
        for _ in range(3):
            r4.step(0)
        el = timed(torch, dist, 1, lambda: r4.step(0), args.steps)
        e4.set_timing(nbd)
        for _ in range(nbd):
            b4.run(stream=cs.cuda_stream)
        torch.cuda.synchronize()
        k4 = e4.kernel_times()
        e4.set_timing(0)
        tot4 = int(b4.total.item())
        other_mix = {"value": round(nbytes * args.steps / el / 2**30, 3),
                     "ms_per_step": round(el / args.steps * 1e3, 4),
                     "params": f"minLen={om_min} pred=(fp&{om_mask:#x})==0 n>minLen"
                               + (" (reference defaults)" if main_is_4k else " (min-variable-segment-size=2)"),
                     "mean_chunk_bytes": round(nbytes / max(tot4, 1), 1), "chunks_per_gpu_step": tot4,
                     "kernels_ms": {k: round(v, 4) for k, v in k4.items() if v}, "records_identical": r4.identical()}
        del r4, b4
        e4.destroy()

    # host paths (rank 0): the batched C-ABI call and the thread sweep of single-buffer calls
    e2e = e2e_pinned = sweep = None
    if rank == 0 and (args.e2e_mib > 0 or args.threads):
        import numpy as np

        nb = min(nbuf, max(args.e2e_mib, 256) * 1024 // args.buf_kib)
        host = batch.data[: nb * buf_len].cpu().numpy()
        if args.e2e_mib > 0:
            offs = np.arange(nb, dtype=np.uint64) * buf_len
            lens = np.full(nb, buf_len, np.uint32)
            eng.chunk_batch(host, offs, lens)  # warm (pinned staging allocation)
            te = time.perf_counter()
            reps = 3
            for _ in range(reps):
                eng.chunk_batch(host, offs, lens)
            e2e = nb * buf_len * reps / (time.perf_counter() - te) / 2**30
            hp = torch.empty(nb * buf_len, dtype=torch.uint8, pin_memory=True)
            hp.copy_(batch.data[: nb * buf_len])
            hpn = hp.numpy()
            eng.chunk_batch(hpn, offs, lens)
            te = time.perf_counter()
            for _ in range(reps):
                eng.chunk_batch(hpn, offs, lens)
            e2e_pinned = nb * buf_len * reps / (time.perf_counter() - te) / 2**30
            del hp, hpn
        if args.threads:
            if args.threads == "auto":
                # SDFS's default write-threads is 3 x availableProcessors (Main.java:211-212): on
                # the GPU box a job's share is its cgroup quota
                q = cpu_quota()
                wt = 3 * int(q if q else min(16, len(os.sched_getaffinity(0))))
                tl = sorted({1, 8, 32, wt, 64, 128, 256})
                tl_other = [1, wt]
            else:
                tl = [int(x) for x in args.threads.split(",") if x]
                tl_other = [1]
            sweep = threads_sweep(cfg, local, host, buf_len, tl, args.threads_mode)
            if other_mix is not None:
                # the other chunk mix's single-buffer latency at 1 thread and at SDFS's default
                # write-threads (the engines of the two mixes differ only in minLen / predicate)
                om_min, om_mask = (4095, 0xFFF) if main_is_4k else (2047, 0x7FF)
                cfg_om = SdfsConfig(chunk_length=buf_len, min_len=om_min, pred_mask=om_mask, hash_type=args.hash_type)
                other_mix["getchunks_threads"] = threads_sweep(cfg_om, local, host, buf_len,
                                                               tl_other, args.threads_mode)

    if rank != 0:
        if dist.is_initialized():
            dist.destroy_process_group()
        return

    value = world * nbytes * args.steps / elapsed / 2**30
    ms_step = elapsed / args.steps * 1e3
    # the roofline's kernel time cannot exceed the step it is part of
    assert 0 < hash_ms_one <= ms_step, f"chunk_hash {hash_ms_one:.3f} ms per launch > {ms_step:.3f} ms per step"
    params = (f"P=0x26CE86126EF863 W=48 minLen={cfg.min_len} maxLen={cfg.max_len} "
              f"pred=(fp&{cfg.pred_mask:#x})==0 n>minLen {args.hash_type}")
    traffic, traffic_src = load_traffic("chunk_hash", params)
    # the CPU restatement on rank 0's host share (the GPU box's CPU share is 16 cores per GPU;
    # the host's nproc shows the whole machine), after all GPU work
    cpu = cpu_baseline_block(args, cfg) if args.cpu_secs > 0 else None
    res = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (counter-based SplitMix64 streams, 0% duplicate), resident in HBM",
        "config": {
            "workload": f"{args.streams} streams x {args.stream_mib} MiB per GPU, CHUNK_LENGTH {buf_len} B "
                        f"({nbuf} buffers, {nbytes / 2**30:.2f} GiB per GPU), fresh CDC state per buffer",
            "params": params,
            "mean_chunk_bytes": round(nbytes / max(total, 1), 1),
            "chunks_per_gpu_step": total,
            "streams_in_flight": nsf,
            "records_identical_across_streams": identical,
            "exchange": (f"RCCL all_gather of 48-B fingerprint records, pipelined ({args.exchange_mode})"
                         if use_ex else "none (N=1)"),
            "exchange_last_step": ex_check,
            "parallelism": f"dp{world} (streams sharded per GPU)",
        },
        "kernels_ms": {k: round(v, 4) for k, v in kt.items()},
        "kernels_note": "every stage: HIP events around each kernel in a separate untimed one-stream pass",
        "roofline": roofline_block(
            nbytes, hash_ms_one, ms_step, sha_blocks, ceiling, traffic, traffic_src,
            "HIP events around chunk_hash on its launch stream over a one-stream timed region of "
            f"{args.steps} steps (stream-ordered: nothing overlaps the kernel)",
            hash_ms_live if nsf >= 2 else None),
        "chunk_hash_ms_per_rank": hash_ms_ranks,
        "exchange_proxy": proxy_info,
        "records_sha256": records_sha,
        "cpu_baseline": cpu,
        ("one_stream" if nsf >= 2 else "two_streams"): other,
        ("at_ref_default" if main_is_4k else "at_4k_mean"): other_mix,
        "e2e_host_gibps": round(e2e, 3) if e2e else None,
        "e2e_pinned_host_gibps": round(e2e_pinned, 3) if e2e_pinned else None,
        "e2e_getchunks_threads": sweep,
        "commit": git_head(),
    }
    print(json.dumps(res), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
