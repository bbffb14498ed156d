"""CPU oracle for LZ4 compression of unique chunks — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and the benches' CPU-baseline legs may import this
module, and only as the checker (or the timed CPU baseline).  The product path (``sdfs_amd``)
never imports it and has no CPU fallback.

* ``compress`` / ``compress_framed`` / ``decompress`` — ctypes binding of ``oracle/lz4_ref.c``,
  the byte-serial restatement of LZ4_compress_generic that lz4-java 1.3.0's native
  fastCompressor runs (CompressionUtils.java:52-53,118-120; HashBlobArchive.java:1281-1289).
* ``system_lz4()`` — the image's own liblz4 (1.9.x), loaded only to PIN the restatement's
  ``V19`` mode byte for byte (and to decode both modes' output independently).  It is not the
  reference (that is r123 inside the absent lz4-java jar) — see lz4_ref.c for the two rules
  in which r123 differs.
* ``text_like`` / ``mixed`` — deterministic compressible inputs (counter-based, no RNG state).
"""
from __future__ import annotations

import ctypes
import ctypes.util

import numpy as np

from . import cdc_oracle as C

R123, V19 = 0, 1
MODES = {"r123": R123, "v19": V19}


def _lib():
    L = C.lib()
    if not getattr(L, "_lz4_bound", False):
        P = ctypes.POINTER
        u8p = P(ctypes.c_uint8)
        L.lz4_ref_bound.argtypes = [ctypes.c_uint32]
        L.lz4_ref_bound.restype = ctypes.c_uint32
        for f in (L.lz4_ref_compress, L.lz4_ref_compress_framed):
            f.argtypes = [ctypes.c_int, u8p, ctypes.c_uint32, u8p, ctypes.c_uint32]
            f.restype = ctypes.c_long
        L.lz4_ref_decompress.argtypes = [u8p, ctypes.c_uint32, u8p, ctypes.c_uint32]
        L.lz4_ref_decompress.restype = ctypes.c_long
        u32p, u64p = P(ctypes.c_uint32), P(ctypes.c_uint64)
        L.lz4_ref_compress_batch.argtypes = [ctypes.c_int, u8p, u64p, u32p, ctypes.c_uint32, u8p, u64p, u32p,
                                             ctypes.c_int]
        L.lz4_ref_compress_batch.restype = ctypes.c_long
        L._lz4_bound = True
    return L


def _arr(data) -> np.ndarray:
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data, np.uint8)
    return np.frombuffer(bytes(data), np.uint8).copy()


def bound(n: int) -> int:
    """LZ4Compressor.maxCompressedLength (LZ4_compressBound)."""
    return n + n // 255 + 16


def compress(data, mode: int = R123) -> bytes:
    a = _arr(data)
    out = np.zeros(bound(len(a)), np.uint8)
    k = _lib().lz4_ref_compress(mode, C._p(a, ctypes.c_uint8), len(a), C._p(out, ctypes.c_uint8), len(out))
    if k < 0:
        raise RuntimeError("lz4_ref_compress failed")
    return out[:k].tobytes()


def compress_framed(data, mode: int = R123) -> bytes:
    """[big-endian int32 len][block]: the chunk record HashBlobArchive.putChunk writes."""
    a = _arr(data)
    out = np.zeros(bound(len(a)) + 4, np.uint8)
    k = _lib().lz4_ref_compress_framed(mode, C._p(a, ctypes.c_uint8), len(a), C._p(out, ctypes.c_uint8), len(out))
    if k < 0:
        raise RuntimeError("lz4_ref_compress_framed failed")
    return out[:k].tobytes()


def compress_batch(base: np.ndarray, offs, lens, mode: int = R123, nthreads: int = 1):
    """Framed records of many chunks on nthreads C threads: (records list, seconds)."""
    import time

    base = np.ascontiguousarray(base, np.uint8)
    offs = np.ascontiguousarray(offs, np.uint64)
    lens = np.ascontiguousarray(lens, np.uint32)
    room = lens.astype(np.uint64) + lens // 255 + 20
    out_offs = np.concatenate([[0], np.cumsum(room)[:-1]]).astype(np.uint64)
    out = np.zeros(int(room.sum()) + 16, np.uint8)
    out_lens = np.zeros(len(lens), np.uint32)
    t0 = time.perf_counter()
    k = _lib().lz4_ref_compress_batch(mode, C._p(base, ctypes.c_uint8), C._p(offs, ctypes.c_uint64),
                                      C._p(lens, ctypes.c_uint32), len(lens), C._p(out, ctypes.c_uint8),
                                      C._p(out_offs, ctypes.c_uint64), C._p(out_lens, ctypes.c_uint32), nthreads)
    secs = time.perf_counter() - t0
    if k < 0:
        raise RuntimeError("lz4_ref_compress_batch failed")
    return [out[int(o): int(o) + int(n)].tobytes() for o, n in zip(out_offs, out_lens)], secs


def system_batch(decompress: bool, base: np.ndarray, offs, lens, out_caps, nthreads: int = 16):
    """The image's liblz4 (oracle/lz4_sys.c, dlopen'd) over many chunks on nthreads C threads:
    LZ4_compress_default (out_caps = room per chunk) or LZ4_decompress_safe (out_caps = decoded
    lengths).  Returns (out, out_offs, out_lens, seconds); the LZ4 bench's CPU legs only."""
    import time

    L = C.fast_lib()
    if not getattr(L, "_lz4_sys_bound", False):
        P = ctypes.POINTER
        u8p, u32p, u64p = P(ctypes.c_uint8), P(ctypes.c_uint32), P(ctypes.c_uint64)
        L.lz4_sys_batch.argtypes = [ctypes.c_int, u8p, u64p, u32p, ctypes.c_uint32, u8p, u64p, u32p, u32p, ctypes.c_int]
        L.lz4_sys_batch.restype = ctypes.c_long
        L._lz4_sys_bound = True
    base = np.ascontiguousarray(base, np.uint8)
    offs = np.ascontiguousarray(offs, np.uint64)
    lens = np.ascontiguousarray(lens, np.uint32)
    caps = np.ascontiguousarray(out_caps, np.uint32)
    out_offs = np.concatenate([[0], np.cumsum(caps.astype(np.uint64))[:-1]]).astype(np.uint64)
    out = np.zeros(int(caps.astype(np.uint64).sum()) + 16, np.uint8)
    out_lens = np.zeros(len(lens), np.uint32)
    t0 = time.perf_counter()
    rc = L.lz4_sys_batch(1 if decompress else 0, C._p(base, ctypes.c_uint8), C._p(offs, ctypes.c_uint64),
                         C._p(lens, ctypes.c_uint32), len(lens), C._p(out, ctypes.c_uint8),
                         C._p(out_offs, ctypes.c_uint64), C._p(caps, ctypes.c_uint32),
                         C._p(out_lens, ctypes.c_uint32), nthreads)
    secs = time.perf_counter() - t0
    if rc != 0:
        raise RuntimeError(f"lz4_sys_batch failed ({rc})")
    return out, out_offs, out_lens, secs


def decompress(block: bytes, n: int) -> bytes:
    a = _arr(block)
    out = np.zeros(max(n, 1), np.uint8)
    k = _lib().lz4_ref_decompress(C._p(a, ctypes.c_uint8), len(a), C._p(out, ctypes.c_uint8), n)
    if k != n:
        raise ValueError(f"lz4_ref_decompress: {k} != {n}")
    return out[:n].tobytes()


# ---------------------------------------------------------------- the image's liblz4 (pin only)
_sys = None


def system_lz4():
    """ctypes handle of the system liblz4 (>= 1.9), or None when the image has none."""
    global _sys
    if _sys is None:
        for name in ("liblz4.so.1", ctypes.util.find_library("lz4") or ""):
            if not name:
                continue
            try:
                L = ctypes.CDLL(name)
            except OSError:
                continue
            L.LZ4_versionNumber.restype = ctypes.c_int
            L.LZ4_compress_default.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
            L.LZ4_compress_default.restype = ctypes.c_int
            L.LZ4_decompress_safe.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
            L.LZ4_decompress_safe.restype = ctypes.c_int
            _sys = L
            break
        else:
            _sys = False
    return _sys or None


def system_compress(data: bytes) -> bytes:
    L = system_lz4()
    out = ctypes.create_string_buffer(bound(len(data)))
    k = L.LZ4_compress_default(bytes(data), out, len(data), len(out))
    if k <= 0 and len(data):
        raise RuntimeError("LZ4_compress_default failed")
    return out.raw[:k]


def system_decompress(block: bytes, n: int) -> bytes:
    L = system_lz4()
    out = ctypes.create_string_buffer(max(n, 1))
    k = L.LZ4_decompress_safe(bytes(block), out, len(block), n)
    if k != n:
        raise ValueError(f"LZ4_decompress_safe: {k} != {n}")
    return out.raw[:n]


# ---------------------------------------------------------------- compressible inputs
_WORDS = [w.encode() for w in (
    "the of and to in is that for it as was with be by on not he this are or his from at which but "
    "have an they you were her she there had one all we can their has been if more when will would "
    "who so no chunk store write buffer file block hash index volume dedup data stream offset length "
    "sdfs archive cloud bucket metadata fingerprint rabin window segment cluster replica").split()]


def text_like(seed: int, stream: int, n: int) -> np.ndarray:
    """Words drawn by a counter-based hash, separated by spaces/newlines: compresses ~2-3x."""
    out = bytearray()
    i = 0
    while len(out) < n:
        h = C.splitmix64((seed * 0x9E3779B97F4A7C15 + stream * 0xD1B54A32D192ED03 + i) & ((1 << 64) - 1))
        out += _WORDS[h % len(_WORDS)]
        out += b"\n" if (h >> 32) % 11 == 0 else b" "
        if (h >> 40) % 37 == 0:
            out += str(h % 100000).encode()
        i += 1
    return np.frombuffer(bytes(out[:n]), np.uint8).copy()


def mixed(seed: int, stream: int, n: int) -> np.ndarray:
    """Random runs, repeats of earlier bytes at short and long distances, zero runs and text."""
    a = np.zeros(n, np.uint8)
    p = 0
    i = 0
    while p < n:
        h = C.splitmix64((seed * 0x9E3779B97F4A7C15 + stream * 0xD1B54A32D192ED03 + (i << 20)) & ((1 << 64) - 1))
        kind = h % 5
        L = int(1 + (h >> 8) % 3000)
        L = min(L, n - p)
        if kind == 0:
            a[p:p + L] = C.synth(seed, stream * 1000 + i, 0, L)
        elif kind == 1 and p > 16:
            d = int(1 + (h >> 24) % min(p, 70000))
            for k in range(L):  # overlapping copy
                a[p + k] = a[p + k - d]
        elif kind == 2:
            a[p:p + L] = 0
        elif kind == 3:
            a[p:p + L] = text_like(seed, stream * 1000 + i, L)
        else:
            a[p:p + L] = (h >> 16) & 0xFF
        p += L
        i += 1
    return a
