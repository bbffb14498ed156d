"""Per-buffer metadata images on the MI355X (include/sdfs_meta.h).

After a batch of write buffers has been chunked (``DeviceBatch`` / ``sdfs_cdc_run_device``) and
deduplicated (``HipHashesMap.put_records``), :func:`emit_map_slots` writes each buffer's
``SparseDataChunk.getBytes()`` image — its ``HashLocPair`` records (SparseDedupFile.java:535-556,
HashLocPair.java:49-59) framed as SparseDataChunk.java:295-318 — into the buffer's
``LongByteArrayMap`` slot (LongByteArrayMap.java:536-579), all on the device.  No CPU fallback.
"""
from __future__ import annotations

import ctypes

from . import _lib
from ._lib import check


def slot_bytes(hash_len: int, chunk_length: int, min_len: int) -> int:
    """LongByteArrayMap slot length of a version >= 2 map (LongByteArrayMap.java:55-60)."""
    return int(_lib.load().sdfs_cdc_map_slot_bytes(hash_len, chunk_length, min_len))


def emit_map_slots(batch, dup, hashloc, hash_len: int = 32, slot_len: int | None = None, device: int = 0,
                   stream=None):
    """batch: a DeviceBatch after run(); dup/hashloc: the index's per-record outputs.
    Returns (map u8 [nbuf * slot_len] zero-initialised then written, doop int32 [nbuf], overflow
    int32 [1]) as device tensors."""
    import torch

    lib = _lib.load()
    cfg = batch.engine.config
    slot_len = slot_len or slot_bytes(hash_len, cfg.chunk_length, cfg.min_len)
    dev = batch.data.device
    m = torch.zeros(batch.nbuf * slot_len, dtype=torch.uint8, device=dev)
    doop = torch.zeros(batch.nbuf, dtype=torch.int32, device=dev)
    ovf = torch.zeros(1, dtype=torch.int32, device=dev)
    s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
    check(lib.sdfs_cdc_map_emit(int(device), batch.nbuf, ctypes.byref(batch.out), int(hash_len), dup.data_ptr(),
                                hashloc.data_ptr(), m.data_ptr(), slot_len, doop.data_ptr(), ovf.data_ptr(), s))
    return m, doop, ovf
