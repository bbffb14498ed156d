"""ctypes binding of tools/libsdfs_threads.so (tools/threads_bench.c): T C threads calling the
engine's getChunks / getHash one buffer at a time, SDFS's flush-thread pattern
(SparseDedupFile.java:100,432; WritableCacheBuffer.java:100-104).  Bench/test infrastructure."""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libsdfs_threads.so")
# linked against the library the engine handles come from (SDFS_CDC_LIB may select the tuning build)
LIB_TUNING = os.path.join(HERE, "libsdfs_threads_tuning.so")


class Result(ctypes.Structure):
    _fields_ = [("secs", ctypes.c_double), ("gibps", ctypes.c_double), ("mean_us", ctypes.c_double),
                ("p50_us", ctypes.c_double), ("p90_us", ctypes.c_double), ("p99_us", ctypes.c_double),
                ("max_us", ctypes.c_double), ("calls", ctypes.c_uint64), ("first_error", ctypes.c_int),
                ("caller_cpu_us", ctypes.c_double), ("fill_us", ctypes.c_double)]

    def as_dict(self) -> dict:
        return {k: (round(getattr(self, k), 3) if isinstance(getattr(self, k), float) else getattr(self, k))
                for k, _ in self._fields_}


_lib = None


def load():
    global _lib
    if _lib is None:
        from sdfs_amd import _lib as engine_lib
        engine_lib.load()  # the engine (and torch's HIP runtime) first
        tuning = os.path.basename(engine_lib.LIB_PATH) == "libsdfs_cdc_tuning.so"
        lib = ctypes.CDLL(LIB_TUNING if tuning else LIB)
        vp = ctypes.c_void_p
        lib.sdfs_threads_getchunks.argtypes = [vp, ctypes.c_int, vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                               ctypes.c_uint32, vp, vp, vp, vp, ctypes.POINTER(Result)]
        lib.sdfs_threads_getchunks_ex.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, ctypes.c_uint64,
                                                  ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32, vp, vp, vp, vp,
                                                  ctypes.POINTER(Result)]
        lib.sdfs_threads_gethash.argtypes = [vp, ctypes.c_int, vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                             ctypes.c_int, vp, ctypes.POINTER(Result)]
        _lib = lib
    return _lib


MODES = {"copy": 0, "fill": 1, "stream": 2}


def getchunks(engine, nthreads: int, data: np.ndarray, buf_len: int, total_calls: int, keep: bool = False,
              engines=None, mode: str = "copy"):
    """data: nbuf * buf_len host bytes.  Returns (Result, results) where results is
    (counts[nbuf], starts[nbuf, cap], lens[nbuf, cap], digests[nbuf, cap, dl]) when keep.
    engines: several engine instances (thread t calls through engines[t % len]); mode: the
    getChunks entry point ("copy" sdfs_cdc_get_chunks, "fill" the JNI glue's
    sdfs_cdc_get_chunks_fill, "stream" sdfs_cdc_get_chunks_stream keyed by buffer // 16)."""
    lib = load()
    engine = engine or engines[0]
    data = np.ascontiguousarray(data, np.uint8)
    nbuf = data.size // buf_len
    cap = engine.slot_cap(buf_len)
    res = Result()
    if keep:
        counts = np.zeros(nbuf, np.uint32)
        st = np.zeros((nbuf, cap), np.uint32)
        ln = np.zeros((nbuf, cap), np.uint32)
        dg = np.zeros((nbuf, cap, engine.digest_len), np.uint8)
        ptrs = (counts.ctypes.data, st.ctypes.data, ln.ctypes.data, dg.ctypes.data)
    else:
        ptrs = (None, None, None, None)
    hs = engines or [engine]
    harr = (ctypes.c_void_p * len(hs))(*[h._h.value for h in hs])
    rc = lib.sdfs_threads_getchunks_ex(harr, len(hs), MODES[mode], nthreads, data.ctypes.data, nbuf, buf_len,
                                       total_calls, cap, *ptrs, ctypes.byref(res))
    if rc:
        raise RuntimeError(f"threads harness failed to start its threads ({rc})")
    return res, ((counts, st, ln, dg) if keep else None)


def gethash(engine, nthreads: int, data: np.ndarray, buf_len: int, total_calls: int, keep: bool = False):
    lib = load()
    data = np.ascontiguousarray(data, np.uint8)
    nbuf = data.size // buf_len
    dg = np.zeros((nbuf, 32), np.uint8)
    res = Result()
    rc = lib.sdfs_threads_gethash(engine._h, nthreads, data.ctypes.data, nbuf, buf_len, total_calls, 1 if keep else 0,
                                  dg.ctypes.data, ctypes.byref(res))
    if rc:
        raise RuntimeError(f"threads harness failed to start its threads ({rc})")
    return res, (dg[:, :engine.digest_len] if keep else None)
