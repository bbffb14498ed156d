"""bench.py end to end in every form the driver can launch: the plain N = 1
line, the in-process device set (--inproc, the N > 1 form without a launcher) and the torchrun
form with the record exchange at one rank.  Each line must parse, carry the roofline (HBM top
level, VALU limiter), the exchange's self-check must hold (every count equals its batch's total,
this rank's rows of the gathered table are its own records), and the exchanged table must be
byte-identical to the plain path's record table (SHA-256 of the bytes).  The CPU, e2e, caller-sweep
and other-mix legs are off: this checks the GPU forms, bench_round_end runs the full line."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
QUICK = ["--steps", "3", "--warmup", "1", "--cpu-secs", "0", "--e2e-mib", "0", "--threads", "",
         "--other-mix", "0", "--ramp-secs", "0.1"]
_lines = {}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(cmd, timeout=420):
    # a child process (never an exec of this GPU-initialised one); its stderr goes to ours
    r = subprocess.run(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=None, text=True, timeout=timeout)
    assert r.returncode == 0, f"{cmd} exited {r.returncode}"
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def _check_line(d, n=1):
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "roofline", "config"):
        assert k in d, k
    assert d["n_gpus"] == n and d["steps"] == 3 and d["value"] > 0
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["limiter"] == "valu" and r["peak"] == 8000.0
    assert 0 < r["kernel_ms"] <= d["ms_per_step"]
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert 0.05 < r["frac"] < 1.0
    assert 0.3 < r["valu"]["frac"] < 1.2


def _plain():
    if "plain" not in _lines:
        _lines["plain"] = _run([sys.executable, "bench.py"] + QUICK)
    return _lines["plain"]


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_bench_plain_n1_line():
    d = _plain()
    _check_line(d)
    assert d["config"]["records_identical_across_streams"] is True
    assert len(d["records_sha256"]) == 64


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_bench_device_set_form_n1():
    d = _run([sys.executable, "bench.py", "--gpus", "1", "--inproc", "1"] + QUICK)
    _check_line(d)
    ex = d["config"]["exchange_last_step"]
    assert ex["counts"] == d["config"]["chunks_per_gpu_step"] and ex["counts_match"] and ex["rows_match"]
    assert len(d["kernels_ms"]["chunk_hash_per_gpu"]) == 1 and d["one_stream"]["value"] > 0
    plain = _plain()
    assert ex["table_sha256"][0] == plain["records_sha256"] == d["records_sha256"]
    # the device-set line is the same work as the headline (3 steps here, so only a loose bound:
    # the full-length lines are 3.5 % apart, profiles/r06/bench/)
    assert d["value"] > 0.8 * plain["value"], (d["value"], plain["value"])


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_bench_torchrun_form_exchange_n1():
    d = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
              "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "1",
              "--exchange", "1"] + QUICK)
    _check_line(d)
    ex = d["config"]["exchange_last_step"]
    assert ex is not None and ex["counts"] == [d["config"]["chunks_per_gpu_step"]]
    assert ex["counts_match"] and ex["rows_match"]
    assert d["chunk_hash_ms_per_rank"] and d["chunk_hash_ms_per_rank"][0] > 0
    plain = _plain()
    assert ex["table_sha256"][0] == plain["records_sha256"] == d["records_sha256"]


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_bench_exchange_proxy_runs():
    d = _run([sys.executable, "bench.py", "--exchange-proxy", "8"] + QUICK)
    _check_line(d)
    p = d["exchange_proxy"]
    assert p["ranks"] == 8 and p["bytes_per_step"] >= 7 * 48 * p["records_per_gpu_step"]
    # paced at --proxy-gbps: alone it lasts at least bytes / rate (longer only if its workgroups
    # cannot copy that fast; the line reports the duration it had)
    want_ms = p["bytes_per_step"] / (p["gbps"] * 1e9) * 1e3
    assert 0.8 * want_ms < p["alone_ms"] < 3.0 * want_ms, (p["alone_ms"], want_ms)
