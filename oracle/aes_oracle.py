"""CPU oracle for AES-CBC chunk encryption — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and the benches' CPU-baseline legs may import this
module, and only as the checker (or the timed CPU baseline).  The product path (``sdfs_amd``)
never imports it and has no CPU fallback.

ctypes binding of ``oracle/aes_ref.c``: the FIPS-197 / SP 800-38A / PKCS#5 restatement of
``EncryptUtils.encryptCBC(chunk, ivspec)`` (EncryptUtils.java:142-152) as
``HashBlobArchive.putChunk`` applies it to the stored record (HashBlobArchive.java:1280-1294).
``key_from_passphrase`` is EncryptUtils.java:47-52 (SHA-256 of the passphrase's bytes).
``openssl_encrypt`` runs the image's ``openssl enc`` CLI — used only to make/pin fixtures.
"""
from __future__ import annotations

import ctypes
import hashlib
import shutil
import subprocess
import time

import numpy as np

from . import cdc_oracle as C


def _lib():
    L = C.lib()
    if not getattr(L, "_aes_bound", False):
        P = ctypes.POINTER
        u8p, u32p, u64p = P(ctypes.c_uint8), P(ctypes.c_uint32), P(ctypes.c_uint64)
        L.aes_ref_cbc_bound.argtypes = [ctypes.c_uint64]
        L.aes_ref_cbc_bound.restype = ctypes.c_uint64
        L.aes_ref_expand_key.argtypes = [u8p, ctypes.c_int, u32p]
        L.aes_ref_expand_key.restype = ctypes.c_int
        for f in (L.aes_ref_encrypt_block, L.aes_ref_decrypt_block):
            f.argtypes = [u32p, ctypes.c_int, u8p, u8p]
            f.restype = None
        L.aes_ref_cbc_encrypt.argtypes = [u8p, ctypes.c_int, u8p, u8p, ctypes.c_int, u8p, ctypes.c_uint64, u8p,
                                          ctypes.c_uint64]
        L.aes_ref_cbc_encrypt.restype = ctypes.c_long
        L.aes_ref_cbc_decrypt.argtypes = [u8p, ctypes.c_int, u8p, u8p, ctypes.c_uint64, u8p, ctypes.c_uint64]
        L.aes_ref_cbc_decrypt.restype = ctypes.c_long
        L.aes_ref_cbc_encrypt_batch.argtypes = [u8p, ctypes.c_int, u8p, u8p, ctypes.c_int, u8p, u64p, u32p,
                                                ctypes.c_uint32, u8p, u64p, u32p, ctypes.c_int]
        L.aes_ref_cbc_encrypt_batch.restype = ctypes.c_long
        L._aes_bound = True
    return L


def _arr(data) -> np.ndarray:
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data, np.uint8)
    return np.frombuffer(bytes(data), np.uint8).copy()


def _u8(a):
    return C._p(a, ctypes.c_uint8)


def bound(n: int) -> int:
    """Cipher.doFinal output length for AES/CBC/PKCS5Padding."""
    return (n // 16 + 1) * 16


def key_from_passphrase(passphrase: str) -> bytes:
    return hashlib.sha256(passphrase.encode()).digest()


def expand_key(key: bytes):
    rk = np.zeros(60, np.uint32)
    nr = _lib().aes_ref_expand_key(_u8(_arr(key)), len(key), C._p(rk, ctypes.c_uint32))
    if nr < 0:
        raise ValueError("AES key must be 16, 24 or 32 bytes")
    return rk, nr


def encrypt_block(key: bytes, block: bytes) -> bytes:
    rk, nr = expand_key(key)
    out = np.zeros(16, np.uint8)
    _lib().aes_ref_encrypt_block(C._p(rk, ctypes.c_uint32), nr, _u8(_arr(block)), _u8(out))
    return out.tobytes()


def decrypt_block(key: bytes, block: bytes) -> bytes:
    rk, nr = expand_key(key)
    out = np.zeros(16, np.uint8)
    _lib().aes_ref_decrypt_block(C._p(rk, ctypes.c_uint32), nr, _u8(_arr(block)), _u8(out))
    return out.tobytes()


def cbc_encrypt(key: bytes, iv: bytes, data, prefix: bytes = b"") -> bytes:
    a, p = _arr(data), _arr(prefix if prefix else b"\0")
    out = np.zeros(bound(len(a) + len(prefix)), np.uint8)
    k = _lib().aes_ref_cbc_encrypt(_u8(_arr(key)), len(key), _u8(_arr(iv)), _u8(p), len(prefix),
                                   _u8(a if len(a) else np.zeros(1, np.uint8)), len(a), _u8(out), len(out))
    if k < 0:
        raise ValueError("aes_ref_cbc_encrypt failed")
    return out[:k].tobytes()


def cbc_decrypt(key: bytes, iv: bytes, data) -> bytes:
    """Raises ValueError on a bad length or padding (Cipher.doFinal's BadPaddingException)."""
    a = _arr(data)
    out = np.zeros(max(len(a), 1), np.uint8)
    k = _lib().aes_ref_cbc_decrypt(_u8(_arr(key)), len(key), _u8(_arr(iv)),
                                   _u8(a if len(a) else np.zeros(1, np.uint8)), len(a), _u8(out), len(out))
    if k < 0:
        raise ValueError("bad padding or length")
    return out[:k].tobytes()


def cbc_encrypt_batch(key: bytes, iv: bytes, base: np.ndarray, offs, lens, prefix: bytes = b"", nthreads: int = 1):
    """Records of many chunks on nthreads C threads: (records list, seconds)."""
    base = np.ascontiguousarray(base, np.uint8)
    offs = np.ascontiguousarray(offs, np.uint64)
    lens = np.ascontiguousarray(lens, np.uint32)
    room = (lens.astype(np.uint64) + len(prefix)) // 16 * 16 + 16
    out_offs = np.concatenate([[0], np.cumsum(room)[:-1]]).astype(np.uint64)
    out = np.zeros(int(room.sum()) + 16, np.uint8)
    out_lens = np.zeros(len(lens), np.uint32)
    p = _arr(prefix if prefix else b"\0")
    t0 = time.perf_counter()
    k = _lib().aes_ref_cbc_encrypt_batch(_u8(_arr(key)), len(key), _u8(_arr(iv)), _u8(p), len(prefix), _u8(base),
                                         C._p(offs, ctypes.c_uint64), C._p(lens, ctypes.c_uint32), len(lens),
                                         _u8(out), C._p(out_offs, ctypes.c_uint64),
                                         C._p(out_lens, ctypes.c_uint32), nthreads)
    secs = time.perf_counter() - t0
    if k < 0:
        raise RuntimeError("aes_ref_cbc_encrypt_batch failed")
    return [out[int(o): int(o) + int(n)].tobytes() for o, n in zip(out_offs, out_lens)], secs


def openssl_encrypt(key: bytes, iv: bytes, data: bytes) -> bytes | None:
    """The image's `openssl enc -aes-{128,192,256}-cbc` (PKCS#7 padding), or None without openssl."""
    exe = shutil.which("openssl")
    if not exe:
        return None
    r = subprocess.run([exe, "enc", f"-aes-{8 * len(key)}-cbc", "-K", key.hex(), "-iv", iv.hex()],
                       input=bytes(data), capture_output=True, check=True)
    return r.stdout
