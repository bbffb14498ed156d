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


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_engine_sharing_and_queue_shutdown_under_tsan(tmp_path):
    """engine_share.h: handles of equal parameters share one engine set (SDFS's many engine
    instances, HashFunctionPool.java:73-86), destroy while calls are in progress waits for them
    (HashFunctionPool.destroyObject, :98-100), calls on a destroyed handle are refused, keyed calls
    stay on their device, unkeyed ones go to the least busy; the queue's shutdown with callers in
    flight completes what was placed and refuses the rest."""
    exe = tmp_path / "share_tsan"
    src = os.path.join(ROOT, "tests", "cpu", "share_tsan.cpp")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-pthread", src, "-o", str(exe)],
                   check=True, timeout=240)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-6000:]
    assert "OK" in r.stdout and "WARNING: ThreadSanitizer" not in r.stderr
