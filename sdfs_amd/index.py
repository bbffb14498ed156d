"""Device-resident dedup-hit index (include/sdfs_index.h) — the step SDFS runs right after
getChunks: group a buffer's chunks by fingerprint, put each distinct one into the hash store
with its claim count, and mark every chunk duplicate or new with its hashloc
(SparseDedupFile.java:435-446,487-564; RocksDBMap.put, RocksDBMap.java:785-870).

:class:`HipHashesMap` mirrors the parts of ``org.opendedup.collections.AbstractHashesMap`` this
step uses (``put`` -> ``InsertRecord``, ``get``, ``containsKey``, ``getSize``, ``getMaxSize``) for a
whole batch of fingerprint records at once.  No CPU fallback: it needs the HIP library and a
gfx950 device.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

from . import _lib


@dataclass
class InsertRecord:
    """org.opendedup.collections.InsertRecord: was the fingerprint inserted, and where it lives."""

    inserted: bool
    pos: int


class HipHashesMap:
    def __init__(self, capacity: int, device: int = 0):
        self._lib = _lib.load()
        h = ctypes.c_void_p()
        _lib.check(self._lib.sdfs_cdc_index_create(int(device), int(capacity), ctypes.byref(h)))
        self._h = h
        self.device = device

    def destroy(self) -> None:
        if self._h:
            self._lib.sdfs_cdc_index_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass

    # --- batch path (device tensors) -------------------------------------------------------
    def put_records(self, records, count=None, pos_base: int = 0, stream=None):
        """Apply fingerprint records (torch uint8 [n, 48] on the device, buffer order).

        ``count``: optional device int32[1] holding the number of valid records (the engine's
        ``total``).  Returns device tensors (dup u8[n], hashloc int64[n], new_list int32[n],
        new_count int64[1]); enqueued on ``stream`` (default: torch's current stream)."""
        import torch

        n = int(records.shape[0])
        dev = records.device
        dup = torch.empty(n, dtype=torch.uint8, device=dev)
        hashloc = torch.empty(n, dtype=torch.int64, device=dev)
        new_list = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        new_count = torch.zeros(1, dtype=torch.int64, device=dev)
        s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
        _lib.check(self._lib.sdfs_cdc_index_put_records(
            self._h, records.data_ptr() if n else None, n, count.data_ptr() if count is not None else None,
            int(pos_base), dup.data_ptr() if n else None, hashloc.data_ptr() if n else None,
            new_list.data_ptr(), new_count.data_ptr(), s))
        return dup, hashloc, new_list, new_count

    def get_digests(self, digests, stream=None):
        """Look up digests (torch uint8 [n, 32] on the device): (pos int64[n], -1 when absent;
        refcount int64[n])."""
        import torch

        n = int(digests.shape[0])
        pos = torch.empty(n, dtype=torch.int64, device=digests.device)
        ref = torch.empty(n, dtype=torch.int64, device=digests.device)
        if n:
            s = stream if stream is not None else torch.cuda.current_stream(digests.device).cuda_stream
            _lib.check(self._lib.sdfs_cdc_index_get(self._h, digests.data_ptr(), n, pos.data_ptr(),
                                                    ref.data_ptr(), s))
        return pos, ref

    # --- AbstractHashesMap-style conveniences (host bytes) -------------------------------------
    def _digest_tensor(self, keys):
        import torch

        buf = bytearray(32 * len(keys))
        for i, k in enumerate(keys):
            if len(k) > 32:
                raise ValueError("fingerprints are at most 32 bytes")
            buf[32 * i:32 * i + len(k)] = k
        return torch.frombuffer(buf, dtype=torch.uint8).reshape(-1, 32).to(f"cuda:{self.device}")

    def get(self, key: bytes) -> int:
        """AbstractHashesMap.get: the fingerprint's pos, or -1."""
        pos, _ = self.get_digests(self._digest_tensor([key]))
        return int(pos[0].item())

    def containsKey(self, key: bytes) -> bool:
        return self.get(key) != -1

    def refcount(self, key: bytes) -> int:
        _, ref = self.get_digests(self._digest_tensor([key]))
        return int(ref[0].item())

    def clear(self, stream=None) -> None:
        """AbstractHashesMap.clear: drop every fingerprint (enqueued on `stream`)."""
        import torch

        s = stream if stream is not None else torch.cuda.current_stream(self.device).cuda_stream
        _lib.check(self._lib.sdfs_cdc_index_clear(self._h, s))

    def getSize(self) -> int:
        used, cap = ctypes.c_uint64(), ctypes.c_uint64()
        _lib.check(self._lib.sdfs_cdc_index_size(self._h, ctypes.byref(used), ctypes.byref(cap)))
        return used.value

    def getMaxSize(self) -> int:
        used, cap = ctypes.c_uint64(), ctypes.c_uint64()
        _lib.check(self._lib.sdfs_cdc_index_size(self._h, ctypes.byref(used), ctypes.byref(cap)))
        return cap.value
