"""Host-side mirror of SDFS's hash-engine plugin surface, bound to the MI355X C-ABI.

The reference host is Java (``org.opendedup.hashing``); no JDK exists in this image, so the host
layer above the C-ABI is restated here with the same names, argument meaning and error behaviour
(the Java/JNI binding a maintainer would add is in INTEGRATION.md):

* :class:`Finger`                       — hashing/Finger.java:32-47 (output record)
* :class:`HipVariableSha256HashEngine`  — implements AbstractHashEngine (AbstractHashEngine.java:24-39)
  like VariableSha256HashEngine (VariableSha256HashEngine.java:39-121), HASH256 / HASH160
* :class:`HipVariableMD5HashEngine`     — like VariableMD5HashEngine (VariableMD5HashEngine.java:37-108)
* :class:`SdfsConfig`                   — the chunking knobs of Main/Config/VolumeConfigWriter
  (Main.java:188-189, Config.java:145-166, VolumeConfigWriter.java:63,96-97,109,298-307)
* :class:`HashFunctionPool`             — hashing/HashFunctionPool.java:29-123 (params + factory + pool)

Every GPU error raises :class:`SdfsCdcError` (an ``IOError``), as ``getChunks`` throws
``IOException`` in the reference.  There is no CPU fallback anywhere in this module.
"""
from __future__ import annotations

import ctypes
import threading
import xml.etree.ElementTree as ET
from collections import deque
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import MD5, MIN_GE, MIN_GT, SHA256, SHA256_160, SdfsCdcError, check

POLY = 10923124345206883  # VariableSha256HashEngine.java:41 / StorageServiceImpl.java:406

VARIABLE_SHA256 = "VARIABLE_SHA256"
VARIABLE_SHA256_160 = "VARIABLE_SHA256_160"
VARIABLE_MD5 = "VARIABLE_MD5"
_ALGO = {VARIABLE_SHA256: SHA256, VARIABLE_SHA256_160: SHA256_160, VARIABLE_MD5: MD5}


@dataclass
class Finger:
    """hashing/Finger.java:32-47 — one chunk of a write buffer."""

    uuid: str | None
    chunk: bytes
    hash: bytes
    start: int
    len: int
    claims: int = -1
    hl: object = None
    ap: int = 0
    noPersist: bool = False


@dataclass
class SdfsConfig:
    """Chunking parameters as SDFS derives them (defaults = mkfs.sdfs defaults).

    ``chunk_length``  Main.CHUNK_LENGTH = chunk-size KiB * 1024 (Config.java:158; 256 KiB default,
                      VolumeConfigWriter.java:63; 40960 KiB with --backup-volume, :304)
    ``min_len``       Main.MIN_CHUNK_LENGTH = min-variable-segment-size KiB * 1024 - 1 (Config.java:145-148;
                      4095, Main.java:189)
    ``max_len``       max-variable-segment-size KiB * 1024 (Config.java:162-166; 32 KiB, 128 KiB backup)
    ``window``        variable-window-size (Config.java:160-161; 48)
    ``hash_type``     hash-type (Config.java:150-151; VARIABLE_SHA256, VolumeConfigWriter.java:109)
    The boundary-predicate knobs are not SDFS settings (the jar's detector is static,
    SURVEY.md A.1); they are exposed because the jar is absent and they are unpinned (A.3):
    ``pred_kind`` PRED_MASK -> ``(fp & pred_mask) == pred_value``, PRED_DIV -> ``fp % pred_div ==
    pred_rem`` (the two detector forms A.3 names).
    """

    chunk_length: int = 256 * 1024
    min_len: int = 4 * 1024 - 1
    max_len: int = 32 * 1024
    window: int = 48
    hash_type: str = VARIABLE_SHA256
    poly: int = POLY
    pred_mask: int = 0xFFF
    pred_value: int = 0
    pred_kind: int = _lib.PRED_MASK  # PRED_DIV: the divisor detector fp % pred_div == pred_rem
    pred_div: int = 0
    pred_rem: int = 0
    min_cmp: int = MIN_GT
    max_batch_bytes: int = 0  # host-batch pinned staging per slot (0 = the engine default, 256 MiB)
    direct: bool = False      # SDFS_CDC_FLAG_DIRECT: one GPU round trip per call (no coalescing)

    @classmethod
    def backup_volume(cls, **kw) -> "SdfsConfig":
        """mkfs.sdfs --backup-volume (VolumeConfigWriter.java:298-307)."""
        kw.setdefault("max_len", 128 * 1024)
        return cls(chunk_length=40960 * 1024, **kw)

    @classmethod
    def from_volume_xml(cls, path: str) -> "SdfsConfig":
        """Parse the ``<io>`` element of a ``*-volume-cfg.xml`` the way Config.parseSDFSConfigFile
        does (Config.java:140-166)."""
        io = ET.parse(path).getroot().find("io")
        if io is None:
            raise ValueError(f"{path}: no <io> element")
        c = cls()
        c.chunk_length = int(io.get("chunk-size")) * 1024
        if io.get("min-variable-segment-size") is not None:
            c.min_len = int(io.get("min-variable-segment-size")) * 1024 - 1
        if io.get("hash-type") is not None:
            c.hash_type = io.get("hash-type")
        if io.get("variable-window-size") is not None:
            c.window = int(io.get("variable-window-size"))
        if io.get("max-variable-segment-size") is not None:
            c.max_len = int(io.get("max-variable-segment-size")) * 1024
        else:
            c.max_len = c.chunk_length  # Config.java:165
        return c

    @property
    def hash_length(self) -> int:
        """HashFunctionPool.hashLength (HashFunctionPool.java:55-64): 32 / 18 (sic) / 16."""
        ht = self.hash_type.upper()
        if ht.startswith("VARIABLE_"):
            if ht.endswith("256"):
                return 32
            if ht.endswith("160"):
                return 18
            return 16
        return 16

    @property
    def max_hash_cluster(self) -> int:
        """HashFunctionPool.max_hash_cluster = CHUNK_LENGTH / minLen (HashFunctionPool.java:66)."""
        return self.chunk_length // self.min_len

    def to_params(self, device: int = 0, hash_type: str | None = None) -> _lib.Params:
        p = _lib.default_params()
        p.poly = self.poly
        p.window = self.window
        p.min_len = self.min_len
        p.max_len = self.max_len
        p.chunk_length = self.chunk_length
        p.pred_mask = self.pred_mask
        p.pred_value = self.pred_value
        p.pred_kind = self.pred_kind
        p.pred_div = self.pred_div
        p.pred_rem = self.pred_rem
        p.min_cmp = self.min_cmp
        p.max_batch_bytes = self.max_batch_bytes
        p.flags = _lib.FLAG_DIRECT if self.direct else 0
        ht = (hash_type or self.hash_type).upper()
        if ht not in _ALGO:
            raise ValueError(f"hash-type {ht} has no variable engine (HashFunctionPool.java:102-121)")
        p.hash_algo = _ALGO[ht]
        p.device = device
        return p


def stream_key(uuid: str) -> int:
    """Stream key of a write stream's uuid (the file GUID getChunks is called with,
    SparseDedupFile.java:432): Java's String.hashCode as an unsigned 32-bit value, which is what
    the JNI glue passes."""
    b = uuid.encode("utf-16-le")
    h = 0
    for i in range(0, len(b), 2):
        h = (31 * h + int.from_bytes(b[i:i + 2], "little")) & 0xFFFFFFFF
    return h


def check_count(rc: int) -> int:
    if rc < 0:
        check(rc)
    return rc


def _buf(data) -> tuple[np.ndarray, int]:
    a = np.frombuffer(data, np.uint8) if isinstance(data, (bytes, bytearray, memoryview)) else np.asarray(data)
    a = np.ascontiguousarray(a, np.uint8)
    return a, a.ctypes.data


class HipVariableSha256HashEngine:
    """AbstractHashEngine on the MI355X (VariableSha256HashEngine.java:39-121)."""

    HASH256 = "HASH256"
    HASH160 = "HASH160"

    def __init__(self, ht: str = HASH256, config: SdfsConfig | None = None, device: int = 0, device_mask: int = 0):
        """device: HIP ordinal, or -1 (ALL_DEVICES) for a device set of every gfx950 GPU;
        device_mask: bit i = ordinal i in the set (overrides device).  Engines with equal
        parameters and device sets share one native engine (include/sdfs_cdc.h "Sharing")."""
        self.config = config or SdfsConfig()
        self.ht = ht
        hash_type = VARIABLE_SHA256_160 if ht == self.HASH160 else self._hash_type()
        self._params = self.config.to_params(device=device, hash_type=hash_type)
        self._params.device_mask = device_mask
        self._lib = _lib.load()
        h = ctypes.c_void_p()
        check(self._lib.sdfs_cdc_create(ctypes.byref(self._params), ctypes.byref(h)))
        self._h = h
        self.digest_len = self._lib.sdfs_cdc_digest_len(h)

    def _hash_type(self) -> str:
        return VARIABLE_SHA256

    # ---- AbstractHashEngine ----
    def isVariableLength(self) -> bool:
        return bool(self._lib.sdfs_cdc_is_variable_length(self._h))

    def getHash(self, data: bytes) -> bytes:
        """VariableSha256HashEngine.getHash (:58-67), computed on the GPU."""
        a, ptr = _buf(data)
        out = (ctypes.c_uint8 * 32)()
        check(self._lib.sdfs_cdc_get_hash(self._h, ptr, len(a), out))
        return bytes(out)[: self.digest_len]

    def getHashes(self, chunks) -> list:
        """getHash over many chunks in one GPU pass (sdfs_cdc_get_hash_batch)."""
        import numpy as np

        chunks = [bytes(c) for c in chunks]
        n = len(chunks)
        if n == 0:
            return []
        lens = np.array([len(c) for c in chunks], np.uint32)
        offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
        base = np.frombuffer(b"".join(chunks) or b"\0", np.uint8)
        out = np.zeros(n * self.digest_len, np.uint8)
        check(self._lib.sdfs_cdc_get_hash_batch(self._h, base.ctypes.data, offs.ctypes.data, lens.ctypes.data, n,
                                                out.ctypes.data))
        return [out[i * self.digest_len:(i + 1) * self.digest_len].tobytes() for i in range(n)]

    def hash_device(self, data, offs, lens, digests, count=None, stream=None) -> None:
        """Device tensors: data u8, offs i64[n], lens i32[n], digests u8[n, 32] (written)."""
        import torch

        n = int(lens.shape[0])
        s = stream if stream is not None else torch.cuda.current_stream(data.device).cuda_stream
        check(self._lib.sdfs_cdc_hash_device(self._h, data.data_ptr(), offs.data_ptr(), lens.data_ptr(),
                                             count.data_ptr() if count is not None else None, n,
                                             digests.data_ptr(), s))

    def setSeed(self, seed: int) -> None:  # no-op in variable engines (:116-120)
        check(self._lib.sdfs_cdc_set_seed(self._h, int(seed)))

    def destroy(self) -> None:
        if getattr(self, "_h", None):
            self._lib.sdfs_cdc_destroy(self._h)
            self._h = None

    def getMaxLen(self) -> int:  # Main.CHUNK_LENGTH (:106-109)
        return self._lib.sdfs_cdc_get_max_len(self._h)

    def getMinLen(self) -> int:  # HashFunctionPool.minLen (:111-114)
        return self._lib.sdfs_cdc_get_min_len(self._h)

    def getChunks(self, data: bytes, uuid: str | None = None) -> list[Finger]:
        """VariableSha256HashEngine.getChunks (:71-86): fresh CDC state per call; returns the
        ordered, contiguous Finger list covering the buffer, each with a copy of its bytes.  The
        uuid names the write stream: on a device set its buffers stay on one GPU."""
        a, ptr = _buf(data)
        starts, lens, digs = self.chunk_arrays(a, stream_key=None if uuid is None else stream_key(uuid))
        raw = a.tobytes()
        return [Finger(uuid, raw[s: s + n], digs[i].tobytes(), int(s), int(n))
                for i, (s, n) in enumerate(zip(starts.tolist(), lens.tolist()))]

    # ---- extensions (batching and arrays) ----
    def slot_cap(self, buf_len: int) -> int:
        return int(self._lib.sdfs_cdc_slot_cap(self._h, buf_len))

    def chunk_arrays(self, data, stream_key: int | None = None,
                     fill: bool = False) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
        """One buffer -> (starts u32[n], lens u32[n], digests u8[n, digest_len]).
        stream_key: the write stream the buffer belongs to (sdfs_cdc_get_chunks_stream: a device
        set keeps one stream on one GPU); fill: hand the bytes over through the fill callback
        (sdfs_cdc_get_chunks_fill, the JNI glue's entry point) instead of a pointer."""
        a, ptr = _buf(data)
        cap = self.slot_cap(max(len(a), 1))
        st = np.zeros(cap, np.uint32)
        ln = np.zeros(cap, np.uint32)
        dg = np.zeros((cap, self.digest_len), np.uint8)
        n = ctypes.c_uint32()
        key = _lib.NO_STREAM if stream_key is None else int(stream_key) & _lib.NO_STREAM
        if fill:
            def _fill(ctx, dst, ln_):
                ctypes.memmove(dst, ptr, ln_)
                return 0

            cb = _lib.FILL_FN(_fill)
            check(self._lib.sdfs_cdc_get_chunks_fill(self._h, key, len(a), cb, None, st.ctypes.data, ln.ctypes.data,
                                                     dg.ctypes.data, cap, ctypes.byref(n)))
        elif stream_key is None:
            check(self._lib.sdfs_cdc_get_chunks(self._h, ptr, len(a), st.ctypes.data, ln.ctypes.data, dg.ctypes.data,
                                                cap, ctypes.byref(n)))
        else:
            check(self._lib.sdfs_cdc_get_chunks_stream(self._h, key, ptr, len(a), st.ctypes.data, ln.ctypes.data,
                                                       dg.ctypes.data, cap, ctypes.byref(n)))
        k = n.value
        return st[:k].copy(), ln[:k].copy(), dg[:k].copy()

    # ---- device set and sharing ----
    def device_count(self) -> int:
        return check_count(self._lib.sdfs_cdc_device_count(self._h))

    def device_ordinals(self) -> list[int]:
        return [check_count(self._lib.sdfs_cdc_device_ordinal(self._h, i)) for i in range(self.device_count())]

    def share_count(self) -> int:
        """Live engine handles sharing this one's native engine (1 = not shared)."""
        return check_count(self._lib.sdfs_cdc_share_count(self._h))

    def chunk_batch(self, base, offs, lens):
        """Many independent buffers (base[offs[b] : offs[b]+lens[b]]) in one GPU pass.
        Returns (counts[nbuf], starts[nbuf, cap], lens[nbuf, cap], digests[nbuf, cap, dl])."""
        a, ptr = _buf(base)
        offs = np.ascontiguousarray(offs, np.uint64)
        lens = np.ascontiguousarray(lens, np.uint32)
        nbuf = len(lens)
        cap = self.slot_cap(int(lens.max()) if nbuf else 1)
        counts = np.zeros(nbuf, np.uint32)
        st = np.zeros((nbuf, cap), np.uint32)
        ln = np.zeros((nbuf, cap), np.uint32)
        dg = np.zeros((nbuf, cap, self.digest_len), np.uint8)
        check(self._lib.sdfs_cdc_get_chunks_batch(self._h, ptr, offs.ctypes.data, lens.ctypes.data, nbuf,
                                                  counts.ctypes.data, st.ctypes.data, ln.ctypes.data,
                                                  dg.ctypes.data, cap))
        return counts, st, ln, dg

    # ---- device-resident path (torch tensors as device memory; no torch in the C-ABI) ----
    def run_device(self, data_ptr: int, nbuf: int, uniform_len: int, out: _lib.DevOut, stream: int = 0,
                   buffer_id_base: int = 0) -> None:
        check(self._lib.sdfs_cdc_run_device(self._h, data_ptr, None, None, nbuf, uniform_len, buffer_id_base,
                                            ctypes.byref(out), stream))

    def run_device_ragged(self, data_ptr: int, data_bytes: int, offs_ptr: int, lens_ptr: int, nbuf: int,
                          out: _lib.DevOut, stream: int = 0, buffer_id_base: int = 0) -> None:
        check(self._lib.sdfs_cdc_run_device_ragged(self._h, data_ptr, data_bytes, offs_ptr, lens_ptr, nbuf,
                                                   buffer_id_base, ctypes.byref(out), stream))

    def synth_device(self, ptr: int, n: int, seed: int, stream_id: int, offset: int = 0, stream: int = 0):
        check(self._lib.sdfs_cdc_synth_device(self._h, ptr, n, seed, stream_id, offset, stream))

    def sync(self) -> None:
        check(self._lib.sdfs_cdc_stream_sync(self._h))

    def queue_timing(self) -> dict:
        """Mean microseconds per coalesced GPU pass: filling, callers' copies, device."""
        f, c, d = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        check(self._lib.sdfs_cdc_queue_timing(self._h, ctypes.byref(f), ctypes.byref(c), ctypes.byref(d)))
        return {"fill_us": round(f.value, 1), "copy_us": round(c.value, 1), "device_us": round(d.value, 1)}

    def queue_early(self) -> int:
        """getChunks calls answered before the rest of their GPU pass finished (cumulative)."""
        n = ctypes.c_uint64()
        check(self._lib.sdfs_cdc_queue_early(self._h, ctypes.byref(n)))
        return n.value

    def queue_stats(self) -> tuple[int, int]:
        """(GPU passes launched, getChunks/getHash calls served) by the coalescing queue."""
        b, r = ctypes.c_uint64(), ctypes.c_uint64()
        check(self._lib.sdfs_cdc_queue_stats(self._h, ctypes.byref(b), ctypes.byref(r)))
        return b.value, r.value

    def set_timing(self, nruns: int) -> None:
        """Record HIP events around every kernel of the next runs (ring of `nruns`; 0 = off)."""
        check(self._lib.sdfs_cdc_set_timing(self._h, int(nruns)))

    STAGES = ("prep", "cdc_scan", "cdc_resolve", "cdc_prefix", "cdc_scatter", "chunk_hash", "pipeline")

    def set_timing_stages(self, nruns: int, stages) -> None:
        """Time only the named stages (fewer events inside a timed region)."""
        mask = 0
        for s in stages:
            mask |= 1 << self.STAGES.index(s)
        check(self._lib.sdfs_cdc_set_timing_mask(self._h, int(nruns), mask))

    def kernel_times(self, dev_index: int = 0) -> dict[str, float]:
        names = (ctypes.c_char_p * 8)()
        ms = (ctypes.c_float * 8)()
        n = self._lib.sdfs_cdc_kernel_times_on(self._h, int(dev_index), names, ms, 8)
        if n < 0:
            check(n)
        return {names[i].decode(): float(ms[i]) for i in range(max(n, 0))}

    def allgather_records(self, records, totals, gathered, streams=None):
        """In-process RCCL all-gather of the device set's fingerprint tables (one entry per set
        member, set order): records[i] u8 [cap_i, 48] and totals[i] (int32/uint32 [1]) on device
        i, gathered[i] u8 [>= n*stride, 48] on device i.  Returns (counts list, stride)."""
        n = len(records)
        rp = (ctypes.c_void_p * n)(*[r.data_ptr() for r in records])
        caps = (ctypes.c_uint64 * n)(*[int(r.numel() // 48) for r in records])
        tp = (ctypes.c_void_p * n)(*[t.data_ptr() for t in totals])
        gp = (ctypes.c_void_p * n)(*[g.data_ptr() for g in gathered])
        gcap = min(int(g.numel() // 48) for g in gathered)
        counts = (ctypes.c_uint32 * n)()
        stride = ctypes.c_uint64()
        sp = (ctypes.c_void_p * n)(*streams) if streams is not None else None
        check(self._lib.sdfs_cdc_allgather_records(self._h, rp, caps, tp, gp, gcap, counts, ctypes.byref(stride), sp))
        return list(counts), int(stride.value)

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


class HipVariableMD5HashEngine(HipVariableSha256HashEngine):
    """VariableMD5HashEngine (VariableMD5HashEngine.java:37-108): same CDC, 16-byte MD5."""

    def __init__(self, config: SdfsConfig | None = None, device: int = 0):
        super().__init__(self.HASH256, config, device)

    def _hash_type(self) -> str:
        return VARIABLE_MD5


class HashFunctionPool:
    """hashing/HashFunctionPool.java: engine factory keyed by hash-type, plus the object pool
    (borrowObject/returnObject, :73-91).  Unknown types return None, as the factory does."""

    def __init__(self, config: SdfsConfig | None = None, device: int = 0):
        self.config = config or SdfsConfig()
        self.device = device
        self._passive: deque = deque()
        self._lock = threading.Lock()

    @property
    def hashLength(self) -> int:
        return self.config.hash_length

    @property
    def max_hash_cluster(self) -> int:
        return self.config.max_hash_cluster

    @property
    def minLen(self) -> int:
        return self.config.min_len

    @property
    def maxLen(self) -> int:
        return self.config.max_len

    @property
    def bytesPerWindow(self) -> int:
        return self.config.window

    def getHashEngine(self):
        ht = self.config.hash_type.upper()
        if ht == VARIABLE_SHA256:
            return HipVariableSha256HashEngine(HipVariableSha256HashEngine.HASH256, self.config, self.device)
        if ht == VARIABLE_SHA256_160:
            return HipVariableSha256HashEngine(HipVariableSha256HashEngine.HASH160, self.config, self.device)
        if ht == VARIABLE_MD5:
            return HipVariableMD5HashEngine(self.config, self.device)
        return None

    def borrowObject(self):
        with self._lock:
            if self._passive:
                return self._passive.popleft()
        return self.getHashEngine()

    def returnObject(self, hc) -> None:
        with self._lock:
            self._passive.append(hc)
