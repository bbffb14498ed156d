"""CPU tests of the engine's host-side concurrency (sdfs_amd/csrc/host_queue.h) under
ThreadSanitizer: the coalescing queue that serves concurrent getChunks/getHash callers on one
shared engine (SparseDedupFile.java:100,432; flush pools WritableCacheBuffer.java:100-104) and
the copy pool of the batched host path, driven by a CPU stand-in backend (no GPU)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_queue_and_copy_pool_under_tsan(tmp_path):
    exe = tmp_path / "queue_tsan"
    src = os.path.join(ROOT, "tests", "cpu", "queue_tsan.cpp")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-pthread", src, "-o", str(exe)],
                   check=True, timeout=240)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-6000:]
    assert "OK" in r.stdout and "WARNING: ThreadSanitizer" not in r.stderr
