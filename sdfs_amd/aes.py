"""AES-CBC of stored chunk records on the MI355X (include/sdfs_aes.h).

Mirrors ``org.opendedup.util.EncryptUtils`` as ``HashBlobArchive`` uses it: with
``chunk-store-encrypt`` on, every stored record ``[int nz][chunk | LZ4 block]`` is passed through
``EncryptUtils.encryptCBC(record, ivspec)`` (HashBlobArchive.java:1280-1294) — JCE
``AES/CBC/PKCS5Padding`` under ``key = SHA-256(passphrase.getBytes())`` (EncryptUtils.java:47-52)
and the archive's 16-byte IV — and read back with ``decryptCBC`` (HashBlobArchive.java:1923-1925).

* :class:`HipEncryptUtils` — ``encryptCBC`` / ``decryptCBC`` on byte strings, plus the batch forms
  the GPU is for: host record lists and device-resident records (e.g. the framed LZ4 output of
  :class:`sdfs_amd.lz4.HipLz4Compressor`), optionally framing raw chunks as ``[int -1][chunk]``
  on the fly.
* :func:`key_from_passphrase` — EncryptUtils' key derivation (host control logic, once).

No CPU fallback: every call runs the HIP kernels and raises :class:`SdfsCdcError` on failure.
``decryptCBC`` retries a record whose padding is bad under the legacy key SHA-256("Password") and
raises ``IOError`` only if that fails too, as ``EncryptUtils.decryptCBC`` does
(EncryptUtils.java:50-52,131-149); the device form does the same for the records that fail when
``legacy_fallback`` is set (a second GPU pass over just those records).
"""
from __future__ import annotations

import ctypes
import hashlib

import numpy as np

from . import _lib
from ._lib import check

BAD_PADDING = 0xFFFFFFFF
# EncryptUtils.oldKeyBytes = getSHAHashBytes("Password".getBytes()) (EncryptUtils.java:50): the key of
# chunk stores written before the passphrase became configurable; decryptCBC falls back to it
LEGACY_KEY = hashlib.sha256(b"Password").digest()


def key_from_passphrase(passphrase: str) -> bytes:
    """HashFunctions.getSHAHashBytes(passphrase.getBytes()) (EncryptUtils.java:49)."""
    return hashlib.sha256(passphrase.encode()).digest()


def cbc_bound(n: int) -> int:
    """Cipher.doFinal output length for n plaintext bytes (PKCS#5 always pads)."""
    return (n // 16 + 1) * 16


def _u8(data) -> np.ndarray:
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data, np.uint8)
    return np.frombuffer(bytes(data), np.uint8)


class HipEncryptUtils:
    """EncryptUtils with a fixed key on one GPU.  iv: the archive's 16 bytes (ivspec)."""

    def __init__(self, key: bytes, device: int = 0):
        if len(key) not in (16, 24, 32):
            raise ValueError("AES key must be 16, 24 or 32 bytes")
        self._lib = _lib.load()
        h = ctypes.c_void_p()
        k = _u8(key)
        check(self._lib.sdfs_cdc_aes_create(int(device), k.ctypes.data, len(k), ctypes.byref(h)))
        self._h = h
        self.device = device
        self._key = bytes(k)
        self._legacy = None  # engine under LEGACY_KEY, created on the first record that needs it

    def _legacy_engine(self) -> "HipEncryptUtils | None":
        if self._key == LEGACY_KEY:
            return None
        if self._legacy is None:
            self._legacy = HipEncryptUtils(LEGACY_KEY, self.device)
        return self._legacy

    @classmethod
    def from_passphrase(cls, passphrase: str, device: int = 0) -> "HipEncryptUtils":
        return cls(key_from_passphrase(passphrase), device)

    def destroy(self) -> None:
        if getattr(self, "_legacy", None) is not None:
            self._legacy.destroy()
            self._legacy = None
        if getattr(self, "_h", None):
            self._lib.sdfs_cdc_aes_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass

    @staticmethod
    def _iv(iv) -> np.ndarray:
        a = _u8(iv)
        if len(a) != 16:
            raise ValueError("IV must be 16 bytes")
        return a

    # ---- EncryptUtils
    def encryptCBC(self, chunk, iv, nz_prefix: int | None = None) -> bytes:
        """EncryptUtils.encryptCBC(chunk, ivspec).  nz_prefix: encrypt [BE int nz_prefix][chunk]
        (the putChunk record) without building it on the host first."""
        a, v = _u8(chunk), self._iv(iv)
        plen = 0 if nz_prefix is None else 4
        cap = cbc_bound(len(a) + plen)
        out = np.zeros(cap, np.uint8)
        n = ctypes.c_uint64()
        check(self._lib.sdfs_cdc_aes_encrypt(self._h, a.ctypes.data if len(a) else None, len(a), plen,
                                             int(nz_prefix or 0), v.ctypes.data, out.ctypes.data, cap,
                                             ctypes.byref(n)))
        return out[: n.value].tobytes()

    def _decrypt_one(self, a: np.ndarray, v: np.ndarray) -> int | bytes:
        out = np.zeros(len(a), np.uint8)
        n = ctypes.c_uint64()
        rc = self._lib.sdfs_cdc_aes_decrypt(self._h, a.ctypes.data, len(a), v.ctypes.data, out.ctypes.data,
                                            len(a), ctypes.byref(n))
        return out[: n.value].tobytes() if rc == _lib.OK else rc

    def decryptCBC(self, enc, iv) -> bytes:
        """EncryptUtils.decryptCBC(encChunk, ivspec) (EncryptUtils.java:131-149): bad padding under
        the configured key -> retry under the legacy key; IOError if both fail."""
        a, v = _u8(enc), self._iv(iv)
        if len(a) == 0 or len(a) % 16:
            raise IOError("ciphertext length is not a positive multiple of 16")
        r = self._decrypt_one(a, v)
        if isinstance(r, bytes):
            return r
        legacy = self._legacy_engine() if r == _lib.EINVAL else None  # EINVAL = bad padding
        if legacy is not None:
            r2 = legacy._decrypt_one(a, v)
            if isinstance(r2, bytes):
                return r2
        check(r)  # SdfsCdcError is an IOError
        raise IOError("decryption failed")

    # ---- batches
    def encrypt_chunks(self, base, offs, lens, iv, nz_prefix: int | None = None) -> list[bytes]:
        """Records base[offs[i] : offs[i]+lens[i]] (each framed as [BE nz_prefix][chunk] when
        nz_prefix is given) in one GPU pass."""
        a = _u8(base)
        offs = np.ascontiguousarray(offs, np.uint64)
        lens = np.ascontiguousarray(lens, np.uint32)
        n = len(lens)
        if n == 0:
            return []
        plen = 0 if nz_prefix is None else 4
        room = (lens.astype(np.uint64) + plen) // 16 * 16 + 16
        out_offs = np.concatenate([[0], np.cumsum(room)[:-1]]).astype(np.uint64)
        out = np.zeros(int(room.sum()) + 16, np.uint8)
        out_lens = np.zeros(n, np.uint32)
        v = self._iv(iv)
        check(self._lib.sdfs_cdc_aes_encrypt_batch(self._h, a.ctypes.data if len(a) else out.ctypes.data,
                                                   offs.ctypes.data, lens.ctypes.data, n, plen, int(nz_prefix or 0),
                                                   v.ctypes.data, out.ctypes.data, out_offs.ctypes.data,
                                                   out_lens.ctypes.data))
        return [out[int(o): int(o) + int(k)].tobytes() for o, k in zip(out_offs, out_lens)]

    def encrypt_device(self, data, src_off, src_len, out, dst_off, dst_len, iv=None, ivs=None, count=None,
                       nz_prefix: int | None = None, stream=None) -> None:
        """Device tensors: data u8, src_off i64[n], src_len i32[n], out u8, dst_off i64[n] (room
        cbc_bound(len + plen) each), dst_len i32[n] (written); iv: 16 host bytes for every record,
        or ivs: device u8[n, 16]; count: optional device int32[1]."""
        import torch

        n = int(src_len.shape[0])
        s = stream if stream is not None else torch.cuda.current_stream(data.device).cuda_stream
        v = self._iv(iv) if iv is not None else None
        check(self._lib.sdfs_cdc_aes_encrypt_device(
            self._h, data.data_ptr(), src_off.data_ptr(), src_len.data_ptr(),
            count.data_ptr() if count is not None else None, n, 0 if nz_prefix is None else 4, int(nz_prefix or 0),
            v.ctypes.data if v is not None else None, ivs.data_ptr() if ivs is not None else None, out.data_ptr(),
            dst_off.data_ptr(), dst_len.data_ptr(), s))

    def decrypt_device(self, data, src_off, src_len, out, dst_off, dst_len, iv=None, ivs=None, count=None,
                       stream=None, legacy_fallback: bool = False) -> None:
        """Inverse of encrypt_device; dst_len[i] = plaintext length or 0xFFFFFFFF (bad padding).
        legacy_fallback: records with bad padding are decrypted again under the legacy key
        (EncryptUtils.decryptCBC's retry) in a second pass over just those records; this waits
        for the first pass on the host to find them."""
        import torch

        n = int(src_len.shape[0])
        s = stream if stream is not None else torch.cuda.current_stream(data.device).cuda_stream
        v = self._iv(iv) if iv is not None else None
        check(self._lib.sdfs_cdc_aes_decrypt_device(
            self._h, data.data_ptr(), src_off.data_ptr(), src_len.data_ptr(),
            count.data_ptr() if count is not None else None, n, v.ctypes.data if v is not None else None,
            ivs.data_ptr() if ivs is not None else None, out.data_ptr(), dst_off.data_ptr(), dst_len.data_ptr(), s))
        legacy = self._legacy_engine() if legacy_fallback else None
        if legacy is None or n == 0:
            return
        st = torch.cuda.ExternalStream(s, device=data.device) if not isinstance(s, torch.cuda.Stream) else s
        with torch.cuda.stream(st):
            live = torch.arange(n, device=dst_len.device)
            if count is not None:
                live = live[live < count.to(torch.int64).reshape(())]
            bad = live[dst_len.view(torch.int32)[live] == -1]  # 0xFFFFFFFF
            k = int(bad.numel())  # host sync: the retry needs the failed records' count
            if k == 0:
                return
            sub_off, sub_len, sub_dst = src_off[bad].contiguous(), src_len[bad].contiguous(), dst_off[bad].contiguous()
            sub_ivs = ivs[bad].contiguous() if ivs is not None else None
            sub_out_len = torch.empty_like(sub_len)
            legacy.decrypt_device(data, sub_off, sub_len, out, sub_dst, sub_out_len, iv=iv, ivs=sub_ivs,
                                  stream=st.cuda_stream)
            dst_len[bad] = sub_out_len.to(dst_len.dtype)
