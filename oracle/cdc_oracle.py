"""CPU oracle for the SDFS variable-block CDC + fingerprint path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker (or the timed CPU baseline).  The product path
(``sdfs_amd``) never imports it and has no CPU fallback.

Three independent restatements live here and are cross-checked by ``tests/test_oracle.py``:

* ``C`` — ctypes binding of ``oracle/libcdc_ref.so`` (``oracle/cdc_ref.c``): scalar C, mirrors the
  reference control flow (VariableSha256HashEngine.getChunks, VariableSha256HashEngine.java:71-86,
  driving the rabinwindow-1.0.2 EnhancedFingerFactory loop).
* ``py_chunk`` — the same loop in pure Python (small inputs only), hashing with ``hashlib``.
* ``gf2_window_fp`` — the definitional GF(2) window fingerprint ``(sum_j b[k-j] x^(8j)) mod P`` with
  Python big ints, independent of any table (SURVEY.md A.2 "equivalent definition").

Parity status: digests are pinned by FIPS 180-4 / RFC 1321 vectors and by the reference's own
blank-chunk constants; boundary rules are **parity unpinned** (the rabinwindow jar is absent and
no reference test pins boundaries — SURVEY.md 8(c)).
"""
from __future__ import annotations

import ctypes
import hashlib
import os
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libcdc_ref.so")
FAST_LIB_PATH = os.path.join(HERE, "libcdc_fast.so")  # cdc_fast.c: bench.py's CPU baseline

SHA256, SHA256_160, MD5 = 0, 1, 2
MIN_GT, MIN_GE = 0, 1
PRED_MASK, PRED_DIV = 0, 1  # bitmask / divisor boundary detector
DIGEST_LEN = {SHA256: 32, SHA256_160: 20, MD5: 16}

POLY = 10923124345206883  # VariableSha256HashEngine.java:41, StorageServiceImpl.java:406
SYNTH_SEED = 0x5DF50001


class CdcRefParams(ctypes.Structure):
    _fields_ = [
        ("poly", ctypes.c_uint64),
        ("window", ctypes.c_uint32),
        ("min_len", ctypes.c_uint32),
        ("max_len", ctypes.c_uint32),
        ("min_cmp", ctypes.c_uint32),
        ("pred_mask", ctypes.c_uint64),
        ("pred_value", ctypes.c_uint64),
        ("hash_algo", ctypes.c_uint32),
        ("pred_kind", ctypes.c_uint32),
        ("pred_div", ctypes.c_uint64),
        ("pred_rem", ctypes.c_uint64),
    ]


@dataclass
class Params:
    """The knobs of SURVEY.md A.1/A.3 (defaults = reference defaults / most likely jar behaviour)."""

    poly: int = POLY
    window: int = 48
    min_len: int = 4095
    max_len: int = 32768
    min_cmp: int = MIN_GT
    pred_mask: int = 0xFFF
    pred_value: int = 0
    hash_algo: int = SHA256
    pred_kind: int = PRED_MASK  # PRED_DIV: fp % pred_div == pred_rem instead of the bitmask form
    pred_div: int = 0
    pred_rem: int = 0

    def to_c(self) -> CdcRefParams:
        return CdcRefParams(self.poly, self.window, self.min_len, self.max_len, self.min_cmp,
                            self.pred_mask, self.pred_value, self.hash_algo, self.pred_kind,
                            self.pred_div, self.pred_rem)

    def is_boundary(self, fp):
        """The boundary predicate on one fingerprint (int) or an array of them."""
        if self.pred_kind == PRED_DIV:
            if isinstance(fp, np.ndarray):
                return (fp % np.uint64(self.pred_div)) == np.uint64(self.pred_rem)
            return fp % self.pred_div == self.pred_rem
        if isinstance(fp, np.ndarray):
            return (fp & np.uint64(self.pred_mask)) == np.uint64(self.pred_value)
        return (fp & self.pred_mask) == self.pred_value

    @property
    def digest_len(self) -> int:
        return DIGEST_LEN[self.hash_algo]

    def slot_cap(self, buf_len: int) -> int:
        shortest = max(1, min(self.min_len + (1 if self.min_cmp == MIN_GT else 0), self.max_len))
        return buf_len // shortest + 2


BACKUP = dict(max_len=131072)  # VolumeConfigWriter.java:298-307 (--backup-volume)


_lib = None


def lib():
    """Load oracle/libcdc_ref.so (built by `make -C oracle` / __graft_entry__.build())."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"oracle library missing: {LIB_PATH} (run `make -C oracle`)")
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.POINTER
        u8p, u32p, u64p = P(ctypes.c_uint8), P(ctypes.c_uint32), P(ctypes.c_uint64)
        L.cdc_ref_tables.argtypes = [ctypes.c_uint64, ctypes.c_uint32, u64p, u64p]
        L.cdc_ref_window_fps.argtypes = [ctypes.c_uint64, ctypes.c_uint32, u8p, ctypes.c_size_t, u64p]
        L.cdc_ref_sha256.argtypes = [u8p, ctypes.c_size_t, u8p]
        L.cdc_ref_md5.argtypes = [u8p, ctypes.c_size_t, u8p]
        L.cdc_ref_hash.argtypes = [ctypes.c_uint32, u8p, ctypes.c_size_t, u8p]
        L.cdc_ref_chunk.argtypes = [P(CdcRefParams), u8p, ctypes.c_size_t, u32p, u32p, u8p, ctypes.c_size_t]
        L.cdc_ref_chunk.restype = ctypes.c_long
        L.cdc_ref_chunk_batch.argtypes = [P(CdcRefParams), u8p, u64p, u32p, ctypes.c_uint32, u32p, u32p,
                                          u32p, u8p, ctypes.c_uint32, ctypes.c_int]
        L.cdc_ref_chunk_batch.restype = ctypes.c_long
        L.cdc_ref_bench_synth.argtypes = [P(CdcRefParams), ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                          ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, u64p, u64p]
        L.cdc_ref_bench_synth.restype = ctypes.c_double
        L.cdc_ref_splitmix64.argtypes = [ctypes.c_uint64]
        L.cdc_ref_splitmix64.restype = ctypes.c_uint64
        L.cdc_ref_synth.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, u8p, ctypes.c_size_t]
        _lib = L
    return _lib


def _p(a: np.ndarray, ct):
    return a.ctypes.data_as(ctypes.POINTER(ct))


_fast = None


def fast_lib():
    """oracle/libcdc_fast.so: the table-driven loop + OpenSSL SHA-256/MD5 (CPU baseline form)."""
    global _fast
    if _fast is None:
        lib()  # its dependency libcdc_ref.so first
        L = ctypes.CDLL(FAST_LIB_PATH)
        P = ctypes.POINTER
        u8p, u32p, u64p = P(ctypes.c_uint8), P(ctypes.c_uint32), P(ctypes.c_uint64)
        L.cdc_fast_chunk.argtypes = [P(CdcRefParams), u8p, ctypes.c_size_t, u32p, u32p, u8p, ctypes.c_size_t]
        L.cdc_fast_chunk.restype = ctypes.c_long
        L.cdc_fast_bench_synth.argtypes = [P(CdcRefParams), ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                           ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, u64p, u64p]
        L.cdc_fast_bench_synth.restype = ctypes.c_double
        _fast = L
    return _fast


def chunk_fast(data: bytes | np.ndarray, p: Params | None = None):
    """cdc_fast_chunk: same contract as chunk() (checked against it in tests/test_oracle.py)."""
    p = p or Params()
    a = np.ascontiguousarray(np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data,
                             np.uint8)
    cap = p.slot_cap(len(a))
    st = np.zeros(cap, np.uint32)
    ln = np.zeros(cap, np.uint32)
    dg = np.zeros((cap, p.digest_len), np.uint8)
    cp = p.to_c()
    n = fast_lib().cdc_fast_chunk(ctypes.byref(cp), _p(a, ctypes.c_uint8), len(a), _p(st, ctypes.c_uint32),
                                  _p(ln, ctypes.c_uint32), _p(dg, ctypes.c_uint8), cap)
    if n < 0:
        raise RuntimeError("cdc_fast_chunk failed")
    return st[:n].copy(), ln[:n].copy(), dg[:n].copy()


def bench_fast(p: Params, nbuf: int, buf_len: int, nthreads: int, seed: int = SYNTH_SEED,
               stream0: int = 0, buffers_per_stream: int = 256):
    """CPU baseline (fast form): returns (seconds, chunks, bytes) for chunk+hash of nbuf buffers."""
    ch = ctypes.c_uint64()
    by = ctypes.c_uint64()
    cp = p.to_c()
    secs = fast_lib().cdc_fast_bench_synth(ctypes.byref(cp), seed, stream0, buffers_per_stream, nbuf, buf_len,
                                           nthreads, ctypes.byref(ch), ctypes.byref(by))
    return secs, ch.value, by.value


# ---------------------------------------------------------------- C oracle wrappers
def tables(poly: int = POLY, window: int = 48):
    push = np.zeros(512, np.uint64)
    pop = np.zeros(256, np.uint64)
    if lib().cdc_ref_tables(poly, window, _p(push, ctypes.c_uint64), _p(pop, ctypes.c_uint64)) != 0:
        raise ValueError("bad polynomial")
    return push, pop


def window_fps(data: bytes | np.ndarray, poly: int = POLY, window: int = 48) -> np.ndarray:
    a = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data
    a = np.ascontiguousarray(a, np.uint8)
    out = np.zeros(len(a), np.uint64)
    lib().cdc_ref_window_fps(poly, window, _p(a, ctypes.c_uint8), len(a), _p(out, ctypes.c_uint64))
    return out


def hash_bytes(data: bytes | np.ndarray, algo: int = SHA256) -> bytes:
    a = np.ascontiguousarray(np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data,
                             np.uint8)
    out = np.zeros(32, np.uint8)
    lib().cdc_ref_hash(algo, _p(a, ctypes.c_uint8), len(a), _p(out, ctypes.c_uint8))
    return out[: DIGEST_LEN[algo]].tobytes()


def chunk(data: bytes | np.ndarray, p: Params | None = None):
    """getChunks restated: returns (starts, lens, digests[n, dl]) as numpy arrays."""
    p = p or Params()
    a = np.ascontiguousarray(np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else data,
                             np.uint8)
    cap = p.slot_cap(len(a))
    st = np.zeros(cap, np.uint32)
    ln = np.zeros(cap, np.uint32)
    dg = np.zeros((cap, p.digest_len), np.uint8)
    cp = p.to_c()
    n = lib().cdc_ref_chunk(ctypes.byref(cp), _p(a, ctypes.c_uint8), len(a), _p(st, ctypes.c_uint32),
                            _p(ln, ctypes.c_uint32), _p(dg, ctypes.c_uint8), cap)
    if n < 0:
        raise RuntimeError("cdc_ref_chunk failed")
    return st[:n].copy(), ln[:n].copy(), dg[:n].copy()


def chunk_batch(base: np.ndarray, offs, lens, p: Params | None = None, nthreads: int = 1):
    """Batch of independent buffers; returns (counts, starts[nbuf,cap], lens[nbuf,cap], digests)."""
    p = p or Params()
    offs = np.ascontiguousarray(offs, np.uint64)
    lens = np.ascontiguousarray(lens, np.uint32)
    nbuf = len(lens)
    cap = p.slot_cap(int(lens.max()) if nbuf else 1)
    counts = np.zeros(nbuf, np.uint32)
    st = np.zeros((nbuf, cap), np.uint32)
    ln = np.zeros((nbuf, cap), np.uint32)
    dg = np.zeros((nbuf, cap, p.digest_len), np.uint8)
    cp = p.to_c()
    base = np.ascontiguousarray(base, np.uint8)
    n = lib().cdc_ref_chunk_batch(ctypes.byref(cp), _p(base, ctypes.c_uint8), _p(offs, ctypes.c_uint64),
                                  _p(lens, ctypes.c_uint32), nbuf, _p(counts, ctypes.c_uint32),
                                  _p(st, ctypes.c_uint32), _p(ln, ctypes.c_uint32), _p(dg, ctypes.c_uint8),
                                  cap, nthreads)
    if n < 0:
        raise RuntimeError("cdc_ref_chunk_batch failed")
    return counts, st, ln, dg


def bench_synth(p: Params, nbuf: int, buf_len: int, nthreads: int, seed: int = SYNTH_SEED,
                stream0: int = 0, buffers_per_stream: int = 256):
    """CPU baseline: returns (seconds, chunks, bytes) for chunk+hash of nbuf synthetic buffers."""
    ch = ctypes.c_uint64()
    by = ctypes.c_uint64()
    cp = p.to_c()
    secs = lib().cdc_ref_bench_synth(ctypes.byref(cp), seed, stream0, buffers_per_stream, nbuf, buf_len,
                                     nthreads, ctypes.byref(ch), ctypes.byref(by))
    return secs, ch.value, by.value


def synth_c(seed: int, stream: int, offset: int, n: int) -> np.ndarray:
    out = np.zeros(n, np.uint8)
    lib().cdc_ref_synth(seed, stream, offset, _p(out, ctypes.c_uint8), n)
    return out


# ---------------------------------------------------------------- synthetic input (numpy)
_M64 = (1 << 64) - 1


def splitmix64_np(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def splitmix64(x: int) -> int:
    z = (x + 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def synth(seed: int, stream: int, offset: int, n: int) -> np.ndarray:
    """Counter-based synthetic bytes: numpy restatement of cdc_ref_synth."""
    key = splitmix64(seed ^ ((stream * 0xD1B54A32D192ED03) & _M64))
    w0 = offset >> 3
    w1 = (offset + n + 7) >> 3
    words = splitmix64_np(np.uint64(key) + np.arange(w0, w1, dtype=np.uint64))
    b = words.view(np.uint8)
    s = offset - (w0 << 3)
    return b[s: s + n].copy()


# ---------------------------------------------------------------- pure-Python restatement
def gf2_mod(v: int, poly: int) -> int:
    d = poly.bit_length() - 1
    while v.bit_length() - 1 >= d:
        v ^= poly << (v.bit_length() - 1 - d)
    return v


def gf2_window_fp(data: bytes, k: int, poly: int = POLY, window: int = 48) -> int:
    """Definition: fp_k = (sum_{j<W, k-j>=0} b[k-j] * x^(8j)) mod P."""
    v = 0
    for j in range(window):
        if k - j < 0:
            break
        v ^= data[k - j] << (8 * j)
    return gf2_mod(v, poly)


def py_tables(poly: int = POLY, window: int = 48):
    d = poly.bit_length() - 1
    push = [(i << d) ^ gf2_mod(i << d, poly) for i in range(512)]
    pop = [gf2_mod(i << (8 * window), poly) for i in range(256)]
    return push, pop


_HASHERS = {
    SHA256: lambda b: hashlib.sha256(b).digest(),
    SHA256_160: lambda b: hashlib.sha256(b).digest()[:20],
    MD5: lambda b: hashlib.md5(b).digest(),
}


def py_chunk(data: bytes, p: Params | None = None):
    """Pure-Python rolling loop; small inputs only.  Returns [(start, len, digest)]."""
    p = p or Params()
    push, pop = py_tables(p.poly, p.window)
    shift = p.poly.bit_length() - 1 - 8
    fp = 0
    ring: list[int] = []
    out = []
    start = n = 0
    h = _HASHERS[p.hash_algo]
    for k, b in enumerate(data):
        fp = ((fp << 8) | b) ^ push[(fp >> shift) & 0x1FF]
        ring.append(b)
        if len(ring) == p.window + 1:
            fp ^= pop[ring.pop(0)]
        n += 1
        min_ok = n >= p.min_len if p.min_cmp == MIN_GE else n > p.min_len
        if (min_ok and p.is_boundary(fp)) or n >= p.max_len:
            out.append((start, n, h(data[start: start + n])))
            start, n = k + 1, 0
    if n > 0:
        out.append((start, n, h(data[start: start + n])))
    return out


def resolve_from_candidates(cand: np.ndarray, length: int, p: Params | None = None):
    """Cut resolution from a candidate bitmap (bool per byte) — the GPU's two-phase formulation
    (candidate scan, then greedy resolve), restated in numpy for cross-checking py_chunk."""
    p = p or Params()
    first_off = p.min_len if p.min_cmp == MIN_GT else max(p.min_len - 1, 0)
    pos = np.flatnonzero(cand[:length])
    out = []
    start = 0
    while start < length:
        lo = start + first_off
        forced = start + p.max_len - 1
        hi = min(forced, length - 1)
        k = -1
        if lo <= hi:
            i = np.searchsorted(pos, lo)
            if i < len(pos) and pos[i] <= hi:
                k = int(pos[i])
        if k < 0:
            k = min(forced, length - 1)
        out.append((start, k + 1 - start))
        start = k + 1
    return out
