"""LZ4 compression of unique chunks on the MI355X (include/sdfs_lz4.h).

Mirrors what SDFS does to a new chunk before it is stored: ``HashBlobArchive.putChunk``
(HashBlobArchive.java:1281-1289) writes ``[int nz, big-endian][CompressionUtils.compressLz4(chunk)]``
when compression is on; ``compressLz4`` is lz4-java 1.3.0's ``LZ4Factory.nativeInstance()
.fastCompressor().compress(byte[])`` (CompressionUtils.java:48-60,118-120).

* :class:`HipLz4Compressor` — ``LZ4Compressor`` (``compress``, ``maxCompressedLength``) plus the
  batch forms the GPU is for: host chunk lists and device-resident chunk extents (e.g. the new
  chunks the dedup index lists after a ``getChunks`` batch).
* :func:`compressLz4` — ``CompressionUtils.compressLz4`` on one chunk.

``mode`` selects the LZ4 release whose bytes are reproduced: ``R123`` (lz4-java 1.3.0's bundled
C LZ4, the reference) or ``V19`` (LZ4 1.9.x ``LZ4_compress_default``).  No CPU fallback: every
call runs the HIP kernels and raises :class:`SdfsCdcError` on failure.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import check

R123, V19 = 0, 1


class HipLz4Compressor:
    def __init__(self, mode: int = R123, device: int = 0):
        self._lib = _lib.load()
        h = ctypes.c_void_p()
        check(self._lib.sdfs_cdc_lz4_create(int(device), int(mode), ctypes.byref(h)))
        self._h = h
        self.mode = mode
        self.device = device

    def destroy(self) -> None:
        if getattr(self, "_h", None):
            self._lib.sdfs_cdc_lz4_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass

    # ---- LZ4Compressor
    def maxCompressedLength(self, n: int) -> int:
        return int(self._lib.sdfs_cdc_lz4_bound(int(n)))

    def compress(self, data) -> bytes:
        """LZ4Compressor.compress(byte[]): one raw LZ4 block."""
        a = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else np.ascontiguousarray(
            data, np.uint8)
        cap = self.maxCompressedLength(len(a))
        out = np.zeros(cap, np.uint8)
        n = ctypes.c_uint32()
        src = a.ctypes.data if len(a) else None
        check(self._lib.sdfs_cdc_lz4_compress(self._h, src, len(a), out.ctypes.data, cap, ctypes.byref(n)))
        return out[: n.value].tobytes()

    # ---- batches
    def compress_chunks(self, base, offs, lens, framed: bool = True) -> list[bytes]:
        """Chunks base[offs[i] : offs[i]+lens[i]] in one GPU pass; framed = the putChunk record."""
        a = np.ascontiguousarray(np.frombuffer(bytes(base), np.uint8) if not isinstance(base, np.ndarray) else base,
                                 np.uint8)
        offs = np.ascontiguousarray(offs, np.uint64)
        lens = np.ascontiguousarray(lens, np.uint32)
        n = len(lens)
        if n == 0:
            return []
        room = lens.astype(np.uint64) + lens // 255 + 16 + (4 if framed else 0)
        out_offs = np.concatenate([[0], np.cumsum(room)[:-1]]).astype(np.uint64)
        out = np.zeros(int(room.sum()) + 16, np.uint8)
        out_lens = np.zeros(n, np.uint32)
        check(self._lib.sdfs_cdc_lz4_compress_batch(self._h, a.ctypes.data if len(a) else out.ctypes.data,
                                                    offs.ctypes.data, lens.ctypes.data, n, out.ctypes.data,
                                                    out_offs.ctypes.data, out_lens.ctypes.data, int(framed)))
        return [out[int(o): int(o) + int(k)].tobytes() for o, k in zip(out_offs, out_lens)]

    def compress_device(self, data, src_off, src_len, out, dst_off, dst_len, count=None, framed: bool = True,
                        stream=None) -> None:
        """Device tensors: data u8, src_off i64[n], src_len i32[n], out u8, dst_off i64[n] (room for
        bound(+4) each), dst_len i32[n] (written); count: optional device int32[1]."""
        import torch

        n = int(src_len.shape[0])
        s = stream if stream is not None else torch.cuda.current_stream(data.device).cuda_stream
        check(self._lib.sdfs_cdc_lz4_compress_device(
            self._h, data.data_ptr(), src_off.data_ptr(), src_len.data_ptr(),
            count.data_ptr() if count is not None else None, n, out.data_ptr(), dst_off.data_ptr(),
            dst_len.data_ptr(), int(framed), s))

    def decompress(self, block, n: int) -> bytes:
        """LZ4FastDecompressor.decompress(src, destLen): IOError (SdfsCdcError) on a malformed block."""
        a = np.frombuffer(bytes(block), np.uint8) if not isinstance(block, np.ndarray) else np.ascontiguousarray(
            block, np.uint8)
        out = np.zeros(max(n, 1), np.uint8)
        check(self._lib.sdfs_cdc_lz4_decompress(self._h, a.ctypes.data if len(a) else None, len(a), out.ctypes.data,
                                                int(n)))
        return out[:n].tobytes()

    def decompress_device(self, data, src_off, src_len, out, dst_off, dst_cap, dst_len, count=None,
                          framed: bool = True, stream=None) -> None:
        """Device tensors: data u8 (blocks or putChunk records), src_off i64[n], src_len i32[n], out u8,
        dst_off i64[n], dst_cap i32[n]; dst_len i32[n] receives the decoded length or -1 (malformed)."""
        import torch

        n = int(src_len.shape[0])
        s = stream if stream is not None else torch.cuda.current_stream(data.device).cuda_stream
        check(self._lib.sdfs_cdc_lz4_decompress_device(
            self._h, data.data_ptr(), src_off.data_ptr(), src_len.data_ptr(),
            count.data_ptr() if count is not None else None, n, out.data_ptr(), dst_off.data_ptr(),
            dst_cap.data_ptr(), dst_len.data_ptr(), int(framed), s))

    def plan_records(self, records, sel=None, count=None, buffer_id_base: int = 0, uniform_len: int = 0,
                     buf_offs=None, framed: bool = True, stream=None):
        """Extents + output offsets of selected 48-byte fingerprint records (device tensors).
        Returns (src_off i64[n], src_len i32[n], dst_off i64[n], total_bytes i64[1])."""
        import torch

        n = int(sel.shape[0]) if sel is not None else int(records.shape[0])
        dev = records.device
        src_off = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        src_len = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        dst_off = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        total = torch.zeros(1, dtype=torch.int64, device=dev)
        s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
        check(self._lib.sdfs_cdc_lz4_plan_records(
            self._h, records.data_ptr() if n else None, sel.data_ptr() if sel is not None and n else None,
            count.data_ptr() if count is not None else None, n, int(buffer_id_base), int(uniform_len),
            buf_offs.data_ptr() if buf_offs is not None else None, int(framed), src_off.data_ptr(),
            src_len.data_ptr(), dst_off.data_ptr(), total.data_ptr(), s))
        return src_off[:n], src_len[:n], dst_off[:n], total


_default = {}


def decompressLz4(data, n: int, device: int = 0) -> bytes:
    """CompressionUtils.decompressLz4(input, len) (CompressionUtils.java:122-125) on the GPU."""
    key = (R123, device)
    if key not in _default:
        _default[key] = HipLz4Compressor(R123, device)
    return _default[key].decompress(data, n)


def compressLz4(data, mode: int = R123, device: int = 0) -> bytes:
    """CompressionUtils.compressLz4 (CompressionUtils.java:118-120) on the GPU."""
    key = (mode, device)
    if key not in _default:
        _default[key] = HipLz4Compressor(mode, device)
    return _default[key].compress(data)
