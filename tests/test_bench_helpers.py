"""CPU tests of bench.py's line helpers (no GPU): the roofline block keeps the contract's HBM
roofline at the top level (bound, peak and frac agree) with the VALU limiter beside it, the
record-table digest is the SHA-256 of the bytes, and the argument parser accepts every form the
driver and the GPU tests launch."""
import hashlib
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_roofline_block_top_level_is_hbm():
    nbytes = 4 << 30
    r = bench.roofline_block(nbytes, 2.7, 3.8, 67_780_347, 1787.0, 6.29e9, "pmc", "src", 4.3)
    assert r["bound"] == "hbm" and r["limiter"] == "valu" and r["unit"] == "GB/s"
    assert r["peak"] == bench.HBM_PEAK_GBPS
    assert r["achieved"] == pytest.approx(nbytes / 2.7e-3 / 1e9, rel=1e-3)
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], abs=1e-4)
    assert r["frac_per_step"] == pytest.approx(nbytes / 3.8e-3 / 1e9 / bench.HBM_PEAK_GBPS, abs=1e-4)
    v = r["valu"]
    assert v["achieved_gbps"] == pytest.approx(67_780_347 * 64 / 2.7e-3 / 1e9, rel=1e-3)
    assert v["frac"] == pytest.approx(v["achieved_gbps"] / 1787.0, abs=1e-3)
    assert r["two_stream_launch_ms"] == 4.3 and r["traffic"] == 6.29e9


def test_table_digest_is_sha256_of_bytes():
    torch = pytest.importorskip("torch")
    t = torch.arange(96, dtype=torch.uint8).view(2, 48)
    assert bench.table_digest(torch, t) == hashlib.sha256(bytes(range(96))).hexdigest()


def test_cli_accepts_the_launch_forms():
    # --help parses every option; the forms themselves need a GPU (tests/test_bench_forms.py)
    r = subprocess.run([sys.executable, "bench.py", "--help"], cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0
    for opt in ("--gpus", "--steps", "--warmup", "--inproc", "--exchange", "--exchange-proxy", "--proxy-wgs",
                "--proxy-gbps", "--proxy-record-bytes", "--proxy-prio", "--threads"):
        assert opt in r.stdout, opt
