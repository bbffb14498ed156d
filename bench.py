#!/usr/bin/env python3
"""bench.py — device-resident GiB/s of variable-block CDC + fingerprint (BASELINE.json metric).

Workload (BASELINE.json configs[1]): per GPU, 64 independent synthetic write
streams x 64 MiB, cut into CHUNK_LENGTH = 256 KiB write buffers (16384 buffers, 4 GiB) resident in
HBM before the timed region; every buffer is chunked from a fresh CDC state with the reference
parameters (P = 0x26CE86126EF863, W = 48, minLen 4095, maxLen 32768, 12-bit predicate, SHA-256).
One step = scan + cut resolution + SHA-256 of every chunk of the 4 GiB; at N > 1 the step also
all-gathers the fingerprint table (48-byte records) over RCCL (sdfs_amd/dist.py).  Weak scaling:
rank r owns streams [64r, 64r+64).

Prints ONE JSON line on rank 0 (contract in the task statement); diagnostics go to stderr.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md); 6.29 TB/s measured float4 copy
VALU_PEAK_OPS = 256 * 4 * 32 * 2.4e9  # 256 CU x 4 SIMD x 32 lanes/clk x 2.4 GHz int32 ops/s
# VALU ops per input byte from the kernels' ISA (DESIGN.md "Roofline"): scan ~11.5, SHA-256 ~21.9
OPS_PER_BYTE = {"cdc_scan": 11.5, "chunk_hash": 21.9}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(target_secs: float, threads: int):
    """The CPU oracle (scalar C restatement, oracle/cdc_ref.c) on a bounded sample of the same
    synthetic workload, timed on this host's cores: a reported baseline, not the target."""
    from oracle import cdc_oracle as O

    p = O.Params()
    t_cal, _, by = O.bench_synth(p, threads * 2, 262144, threads)
    rate = by / max(t_cal, 1e-6)
    nbuf = max(threads * 4, int(rate * target_secs / 262144) // threads * threads)
    secs, chunks, nbytes = O.bench_synth(p, nbuf, 262144, threads, buffers_per_stream=256)
    return dict(value=round(nbytes / secs / 2**30, 4), unit="GiB/s", cores=threads, kind="port",
                sample=f"{nbuf} x 256 KiB synthetic write buffers (streams 0..{(nbuf - 1) // 256}, "
                       f"same generator/params), SHA-256, {threads} threads, {secs:.1f} s, "
                       f"{nbytes / max(chunks, 1):.0f} B mean chunk; CPU restatement, not the Java reference")


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def load_traffic(name: str):
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        return d.get(name, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


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
    ap.add_argument("--e2e-mib", type=int, default=1024, help="host->GPU->host measurement size (0 = skip)")
    ap.add_argument("--min-seg-kib", type=int, default=4,
                    help="min-variable-segment-size (minLen = KiB*1024-1; 4 = the reference default)")
    ap.add_argument("--mask-bits", type=int, default=12,
                    help="boundary predicate (fp & (2^bits-1)) == 0 (12 = the default knob, SURVEY.md A.3)")
    ap.add_argument("--hash-type", default="VARIABLE_SHA256",
                    choices=["VARIABLE_SHA256", "VARIABLE_SHA256_160", "VARIABLE_MD5"])
    ap.add_argument("--ramp-secs", type=float, default=0.3, help="untimed clock ramp before the warmup steps")
    ap.add_argument("--pipelined", type=int, default=1, help="also time two batches in flight (N = 1)")
    ap.add_argument("--exchange", type=int, default=-1,
                    help="record all-gather: -1 = when N > 1, 1 = also at N = 1 (exercises the path)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(local)
    use_ex = world > 1 if args.exchange < 0 else bool(args.exchange)
    if use_ex:
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))

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
    batch = DeviceBatch(eng, nbuf=nbuf, buf_len=buf_len, device=f"cuda:{local}")
    batch.fill_streams(first_stream=streams.start, bufs_per_stream=bufs_per_stream)
    torch.cuda.synchronize()
    cs = torch.cuda.current_stream()
    # N > 1: the one real exchange (all-gather of the fingerprint records), pipelined on a side
    # stream so step i's tables travel while step i+1 is chunked (sdfs_amd/dist.py)
    ex = RecordExchange(batch.recs.view(-1, 48).shape[0], f"cuda:{local}") if use_ex else None
    gathered = [0]

    def step():
        batch.run(buffer_id_base=rank * nbuf, stream=cs.cuda_stream)
        if ex is not None:
            ex.submit(batch.recs.view(-1, 48), batch.total, stream=cs)

    def drain():
        if ex is not None:
            res = ex.flush()
            gathered[0] = sum(cl for _, counts in res[-1:] for cl in counts)

    # clock ramp: ~0.3 s of chunking before the W warmup steps (the GPU idles while the host sets
    # up and its clocks drop; a few 4.5 ms steps do not bring them back), outside the timed region
    t_ramp = time.perf_counter()
    while time.perf_counter() - t_ramp < args.ramp_secs:
        batch.run(buffer_id_base=rank * nbuf, stream=cs.cuda_stream)
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    # timed region: HIP events only around the dominant kernel (the roofline's launch duration),
    # so the per-kernel event pairs of the breakdown do not tax the measured throughput
    eng.set_timing_stages(args.steps, ("chunk_hash",))
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    drain()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], device=f"cuda:{local}", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    hash_ms_live = eng.kernel_times().get("chunk_hash", 0.0)
    # per-stage breakdown (untimed pass, events around every kernel)
    nbd = max(3, min(args.steps, 10))
    eng.set_timing(nbd)
    for _ in range(nbd):
        batch.run(buffer_id_base=rank * nbuf, stream=cs.cuda_stream)
    torch.cuda.synchronize()
    kt = eng.kernel_times()
    eng.set_timing(0)
    kt["chunk_hash"] = hash_ms_live
    counts, _, _, _, total = batch.host_results()

    # two batches in flight (N = 1): a second engine alternates with the first on its own stream,
    # so batch i+1's scan overlaps the tail of batch i's fingerprinting.  Reported beside the
    # value (which stays the one-stream rate the roofline's launch durations describe).
    pipelined = None
    if world == 1 and args.pipelined:
        eng2 = HashFunctionPool(cfg, device=local).getHashEngine()
        batch2 = DeviceBatch(eng2, nbuf=nbuf, buf_len=buf_len, device=f"cuda:{local}")
        batch2.data = batch.data
        ss = [cs, torch.cuda.Stream()]
        pair = [batch, batch2]
        for k in range(2):
            pair[k].run(stream=ss[k].cuda_stream)
        torch.cuda.synchronize()
        tp = time.perf_counter()
        for i in range(args.steps):
            pair[i % 2].run(stream=ss[i % 2].cuda_stream)
        torch.cuda.synchronize()
        el = time.perf_counter() - tp
        same = bool(torch.equal(batch2.record_table(), batch.record_table()))
        pipelined = {"value": round(nbuf * buf_len * args.steps / el / 2**30, 3),
                     "ms_per_step": round(el / args.steps * 1e3, 4), "steps": args.steps,
                     "mode": "2 engines, whole batches alternating on 2 streams", "records_identical": same}
        del batch2
        eng2.destroy()

    # end-to-end (pinned host staging + H2D + kernels + D2H), rank 0 only
    e2e = e2e_pinned = None
    if rank == 0 and args.e2e_mib > 0:
        nb = min(nbuf, args.e2e_mib * 1024 // args.buf_kib)
        host = batch.data[: nb * buf_len].cpu().numpy()
        import numpy as np

        offs = np.arange(nb, dtype=np.uint64) * buf_len
        lens = np.full(nb, buf_len, np.uint32)
        eng.chunk_batch(host, offs, lens)  # warm (pinned staging allocation)
        te = time.perf_counter()
        reps = 3
        for _ in range(reps):
            eng.chunk_batch(host, offs, lens)
        e2e = nb * buf_len * reps / (time.perf_counter() - te) / 2**30
        # the same from pinned host memory (a JNI direct buffer registered with the driver): the
        # engine copies to the GPU straight from it, no staging copy
        hp = torch.empty(nb * buf_len, dtype=torch.uint8, pin_memory=True)
        hp.copy_(batch.data[: nb * buf_len])
        hpn = hp.numpy()
        eng.chunk_batch(hpn, offs, lens)
        te = time.perf_counter()
        for _ in range(reps):
            eng.chunk_batch(hpn, offs, lens)
        e2e_pinned = nb * buf_len * reps / (time.perf_counter() - te) / 2**30
        del hp, hpn

    if rank != 0:
        if use_ex:
            dist.destroy_process_group()
        return

    nbytes = nbuf * buf_len
    value = world * nbytes * args.steps / elapsed / 2**30
    dom = max(("cdc_scan", "chunk_hash"), key=lambda k: kt.get(k, 0.0))
    t_dom = kt.get(dom, 0.0) / 1e3
    achieved = nbytes / t_dom / 1e9 if t_dom > 0 else 0.0
    # device time of one pass: the pipeline-level events when present, else the stage sum
    dev_ms = kt.get("pipeline") or sum(v for k, v in kt.items() if k != "pipeline")
    valu = {k: round(nbytes * OPS_PER_BYTE[k] / (kt[k] / 1e3) / VALU_PEAK_OPS, 3) for k in OPS_PER_BYTE if kt.get(k)}
    cpu = None
    if world == 1 and args.cpu_secs > 0:
        th = args.cpu_threads or min(16, len(os.sched_getaffinity(0)))
        log(f"cpu baseline: {th} threads, ~{args.cpu_secs}s sample")
        cpu = cpu_baseline(args.cpu_secs, th)
        if th > 1 and args.cpu_1t_secs > 0:  # T = all cores and T = 1
            one = cpu_baseline(args.cpu_1t_secs, 1)
            cpu["one_thread"] = {"value": one["value"], "sample": one["sample"]}
        cpu["cpu_model"] = cpu_model()
    res = {
        "metric": "device-resident GiB/s CDC+fingerprint, 4 KiB-mean chunks, 1/2/4/8 MI355X",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (counter-based SplitMix64 streams, 0% duplicate), resident in HBM",
        "config": {
            "workload": f"{args.streams} streams x {args.stream_mib} MiB per GPU, CHUNK_LENGTH {buf_len} B "
                        f"({nbuf} buffers, {nbytes / 2**30:.2f} GiB per GPU), fresh CDC state per buffer",
            "params": f"P=0x26CE86126EF863 W=48 minLen={cfg.min_len} maxLen={cfg.max_len} "
                      f"pred=(fp&{cfg.pred_mask:#x})==0 n>minLen {args.hash_type}",
            "mean_chunk_bytes": round(nbytes / max(total, 1), 1),
            "chunks_per_gpu_step": total,
            "exchange": "RCCL all_gather of 48-B fingerprint records, pipelined" if use_ex else "none (N=1)",
            "parallelism": f"dp{world} (streams sharded per GPU)",
        },
        "kernels_ms": {k: round(v, 4) for k, v in kt.items()},
        "kernels_note": "chunk_hash: HIP events on the launch stream over the timed steps; other stages: a "
                        "separate untimed pass with events around every kernel",
        "roofline": {
            "bound": "hbm",
            "kernel": dom,
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": load_traffic(dom),
            "pipeline_gbps": round(nbytes / (dev_ms / 1e3) / 1e9, 1) if dev_ms else None,
            "valu_frac": valu,
        },
        "cpu_baseline": cpu,
        "e2e_host_gibps": round(e2e, 3) if e2e else None,
        "e2e_pinned_host_gibps": round(e2e_pinned, 3) if e2e_pinned else None,
        "pipelined_2stream": pipelined,
    }
    print(json.dumps(res), flush=True)
    if use_ex:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
