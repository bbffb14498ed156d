"""AES-CBC of stored chunk records (include/sdfs_aes.h).

CPU: the oracle restatement (oracle/aes_ref.c, FIPS-197 in byte form) against the FIPS-197
Appendix C known answers and the NIST SP 800-38A F.2 CBC vectors; the committed fixtures
(tests/golden/aes.json: ciphertexts of the image's `openssl enc`, incl. the putChunk record's
[int nz] prefix and SDFS's SHA-256 key derivation) are reproduced; PKCS#5 padding is checked on
decryption; the library fails loudly without a GPU.
GPU: the HIP cipher, through the C-ABI, against the oracle — single records of every length
class and key size, host batches, the golden fixtures, decryption and bad-padding detection,
the device path with unaligned offsets, per-record IVs and a device count, and the LZ4 -> AES
chain of a compressed, encrypted chunk store.
Parity status: pinned (FIPS/NIST vectors and openssl fixtures)."""
import ctypes
import hashlib
import struct

import numpy as np
import pytest

from oracle import aes_oracle as A
from oracle import cdc_oracle as C
from oracle import lz4_oracle as Z
from sdfs_amd import _lib
from tests import golden_util as G
from tests.golden.make_aes_golden import make_input

FIPS197 = [  # Appendix C.1-C.3: plaintext 00112233..ff, key 000102..
    (16, "69c4e0d86a7b0430d8cdb78070b4c55a"),
    (24, "dda97ca4864cdfe06eaf70a0ec0d7191"),
    (32, "8ea2b7ca516745bfeafc49904b496089"),
]
SP800_38A_PT = ("6bc1bee22e409f96e93d7e117393172a" "ae2d8a571e03ac9c9eb76fac45af8e51"
                "30c81c46a35ce411e5fbc1191a0a52ef" "f69f2445df4f9b17ad2b417be66c3710")
SP800_38A = [  # F.2.1 CBC-AES128.Encrypt, F.2.5 CBC-AES256.Encrypt; IV 000102..0f
    ("2b7e151628aed2a6abf7158809cf4f3c",
     "7649abac8119b246cee98e9b12e9197d" "5086cb9b507219ee95db113a917678b2"
     "73bed6b8e3c1743b7116e69e22229516" "3ff1caa1681fac09120eca307586e1a7"),
    ("603deb1015ca71be2b73aef0857d77811f352c073b6108d72d9810a30914dff4",
     "f58c4c04d6e5f1ba779eabfb5f7bfbd6" "9cfc4e967edb808d679f777bc6702c7d"
     "39f23369a9d9bacfa530e26304231461" "b2eb05e2c39be9fcda6c19078c6a9d1b"),
]
IV0 = bytes(range(16))
LENS = [0, 1, 11, 12, 13, 15, 16, 17, 31, 32, 33, 100, 4095, 4096, 4097, 8191, 32768, 65547, 131072]


def test_oracle_fips197_known_answers():
    pt = bytes.fromhex("00112233445566778899aabbccddeeff")
    for klen, ct in FIPS197:
        key = bytes(range(klen))
        assert A.encrypt_block(key, pt).hex() == ct
        assert A.decrypt_block(key, bytes.fromhex(ct)) == pt


def test_oracle_sp800_38a_cbc_vectors():
    pt = bytes.fromhex(SP800_38A_PT)
    for key, ct in SP800_38A:
        out = A.cbc_encrypt(bytes.fromhex(key), IV0, pt)
        assert out[:64].hex() == ct and len(out) == 80  # PKCS#5 adds a whole block to 64 bytes
        assert A.cbc_decrypt(bytes.fromhex(key), IV0, out) == pt


def test_oracle_reproduces_aes_golden_fixtures():
    fx = G.load("aes.json")["fixtures"]
    assert len(fx) >= 70
    for f in fx:
        data = make_input(f)
        assert hashlib.sha256(data).hexdigest() == f["input_sha256"]
        key, iv = bytes.fromhex(f["key"]), bytes.fromhex(f["iv"])
        if "passphrase" in f:
            assert A.key_from_passphrase(f["passphrase"]) == key
        pre = b"" if f["prefix"] is None else struct.pack(">i", f["prefix"])
        out = A.cbc_encrypt(key, iv, data, prefix=pre)
        assert len(out) == f["out_len"] == A.bound(len(data) + len(pre))
        assert hashlib.sha256(out).hexdigest() == f["out_sha256"]
        if "out_hex" in f:
            assert out.hex() == f["out_hex"]


def test_oracle_padding_checks():
    key = bytes(32)
    ct = A.cbc_encrypt(key, IV0, b"x" * 20)
    assert A.cbc_decrypt(key, IV0, ct) == b"x" * 20
    bad = bytearray(ct)
    bad[-1] ^= 1  # garbles the last block's plaintext, hence its padding
    with pytest.raises(ValueError):
        A.cbc_decrypt(key, IV0, bytes(bad))
    with pytest.raises(ValueError):
        A.cbc_decrypt(key, IV0, ct[:-1])


def test_aes_fails_loudly_without_gpu():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is present")
    except ImportError:
        pass
    L = _lib.load()
    h = ctypes.c_void_p()
    key = (ctypes.c_uint8 * 32)()
    assert L.sdfs_cdc_aes_create(0, key, 32, ctypes.byref(h)) == _lib.ENODEV and not h.value
    assert L.sdfs_cdc_aes_create(0, key, 20, ctypes.byref(h)) == _lib.EINVAL
    assert L.sdfs_cdc_aes_cbc_bound(0) == 16 and L.sdfs_cdc_aes_cbc_bound(16) == 32
    assert L.sdfs_cdc_aes_cbc_bound(4099) == 4112
    from sdfs_amd.aes import HipEncryptUtils
    with pytest.raises(_lib.SdfsCdcError):
        HipEncryptUtils(bytes(32))


# ------------------------------------------------------------------------------------------
# GPU
# ------------------------------------------------------------------------------------------
_CIPH = {}


def ciph(key: bytes):
    from sdfs_amd.aes import HipEncryptUtils
    if key not in _CIPH:
        _CIPH[key] = HipEncryptUtils(key)
    return _CIPH[key]


def _key(klen, k=0):
    return C.synth(77, 500 + k, 0, klen).tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("klen", [16, 24, 32])
def test_gpu_single_records_vs_oracle(klen):
    key = _key(klen)
    c = ciph(key)
    for n in LENS:
        d = C.synth(3, n, 0, n).tobytes()
        iv = C.synth(4, n, 0, 16).tobytes()
        assert c.encryptCBC(d, iv) == A.cbc_encrypt(key, iv, d), n
        pre = struct.pack(">i", -1)
        assert c.encryptCBC(d, iv, nz_prefix=-1) == A.cbc_encrypt(key, iv, d, prefix=pre), n


@pytest.mark.gpu
def test_gpu_known_answers_and_passphrase_key():
    pt = bytes.fromhex(SP800_38A_PT)
    for key, ct in SP800_38A:
        assert ciph(bytes.fromhex(key)).encryptCBC(pt, IV0)[:64].hex() == ct
    from sdfs_amd.aes import HipEncryptUtils, key_from_passphrase
    e = HipEncryptUtils.from_passphrase("Password")
    assert key_from_passphrase("Password") == A.key_from_passphrase("Password")
    d = C.synth(9, 9, 0, 9000).tobytes()
    assert e.encryptCBC(d, IV0) == A.cbc_encrypt(A.key_from_passphrase("Password"), IV0, d)
    e.destroy()


@pytest.mark.gpu
def test_gpu_golden_fixtures():
    fx = G.load("aes.json")["fixtures"]
    by_key = {}
    for f in fx:
        by_key.setdefault((f["key"], f["iv"], f["prefix"]), []).append(f)
    for (key, iv, prefix), group in by_key.items():
        datas = [make_input(f) for f in group]
        offs = np.concatenate([[0], np.cumsum([len(d) + 5 for d in datas[:-1]])]).astype(np.uint64)
        base = np.zeros(int(offs[-1]) + len(datas[-1]) + 8, np.uint8)
        for o, d in zip(offs, datas):
            base[int(o): int(o) + len(d)] = np.frombuffer(d, np.uint8)
        outs = ciph(bytes.fromhex(key)).encrypt_chunks(base, offs, [len(d) for d in datas], bytes.fromhex(iv),
                                                      nz_prefix=prefix)
        for f, out in zip(group, outs):
            assert len(out) == f["out_len"] and hashlib.sha256(out).hexdigest() == f["out_sha256"], f


@pytest.mark.gpu
def test_gpu_batch_and_decrypt_round_trip():
    key = _key(32, 1)
    c = ciph(key)
    rng = np.random.default_rng(11)
    lens = [int(x) for x in rng.integers(0, 40000, 400)] + LENS
    datas = [C.synth(5, i, 0, n).tobytes() for i, n in enumerate(lens)]
    offs = np.concatenate([[0], np.cumsum([len(d) + 7 for d in datas[:-1]])]).astype(np.uint64)
    base = np.zeros(int(offs[-1]) + len(datas[-1]) + 8, np.uint8)
    for o, d in zip(offs, datas):
        base[int(o): int(o) + len(d)] = np.frombuffer(d, np.uint8)
    iv = bytes(range(100, 116))
    outs = c.encrypt_chunks(base, offs, lens, iv, nz_prefix=-1)
    for d, out in zip(datas, outs):
        assert out == A.cbc_encrypt(key, iv, d, prefix=b"\xff\xff\xff\xff")
    for d, out in list(zip(datas, outs))[:60]:
        assert c.decryptCBC(out, iv) == b"\xff\xff\xff\xff" + d
    bad = bytearray(outs[3])
    bad[-1] ^= 0x55
    with pytest.raises(IOError):
        c.decryptCBC(bytes(bad), iv)


@pytest.mark.gpu
def test_gpu_device_path_ivs_count_and_decrypt():
    import torch

    key = _key(32, 2)
    c = ciph(key)
    rng = np.random.default_rng(12)
    n = 3000
    lens = rng.integers(0, 33000, n).astype(np.int64)
    lens[:5] = [0, 1, 15, 16, 17]
    src_off = np.concatenate([[3], 3 + np.cumsum(lens[:-1] + 1)]).astype(np.int64)  # odd, unaligned
    data = C.synth(6, 0, 0, int(src_off[-1] + lens[-1] + 16))
    room = (lens // 16 + 1) * 16
    dst_off = np.concatenate([[5], 5 + np.cumsum(room[:-1] + 3)]).astype(np.int64)
    ivs = C.synth(7, 0, 0, 16 * n).reshape(n, 16)
    dev = torch.device("cuda:0")
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)  # noqa: E731
    d_data, d_soff, d_slen = t(data, torch.uint8), t(src_off, torch.int64), t(lens, torch.int32)
    d_doff, d_ivs = t(dst_off, torch.int64), t(ivs, torch.uint8)
    out = torch.zeros(int(dst_off[-1] + room[-1] + 16), dtype=torch.uint8, device=dev)
    dlen = torch.full((n,), -7, dtype=torch.int32, device=dev)
    k = n - 100  # only the first k records are live (device count)
    cnt = torch.tensor([k], dtype=torch.int32, device=dev)
    c.encrypt_device(d_data, d_soff, d_slen, out, d_doff, dlen, ivs=d_ivs, count=cnt)
    torch.cuda.synchronize()
    o, dl = out.cpu().numpy(), dlen.cpu().numpy()
    assert (dl[k:] == -7).all()
    for i in list(range(0, k, 7)) + [0, 1, 2, 3, 4, k - 1]:
        want = A.cbc_encrypt(key, ivs[i].tobytes(), data[src_off[i]: src_off[i] + lens[i]].tobytes())
        assert dl[i] == len(want) and o[dst_off[i]: dst_off[i] + dl[i]].tobytes() == want, i
    # decrypt the ciphertexts back (device), one corrupted
    ct_len = torch.from_numpy(dl[:k].astype(np.int32)).to(dev)
    o2 = out.clone()
    bad = 17
    o2[int(dst_off[bad] + dl[bad] - 1)] ^= 0x5A
    back = torch.zeros(int(src_off[-1] + lens[-1] + 32), dtype=torch.uint8, device=dev)
    plen = torch.zeros(k, dtype=torch.int32, device=dev)
    c.decrypt_device(o2, d_doff[:k], ct_len, back, d_soff[:k], plen, ivs=d_ivs)
    torch.cuda.synchronize()
    b, pl = back.cpu().numpy(), plen.cpu().numpy().view(np.uint32)
    assert pl[bad] == 0xFFFFFFFF
    for i in range(k):
        if i == bad:
            continue
        assert pl[i] == lens[i], i
        assert b[src_off[i]: src_off[i] + lens[i]].tobytes() == data[src_off[i]: src_off[i] + lens[i]].tobytes(), i


def _oracle_decrypt_with_fallback(key, iv, ct):
    """EncryptUtils.decryptCBC (EncryptUtils.java:131-149): the configured key, then the legacy key."""
    from sdfs_amd.aes import LEGACY_KEY
    for k in (key, LEGACY_KEY):
        try:
            return A.cbc_decrypt(k, iv, ct)
        except ValueError:
            continue
    return None


@pytest.mark.gpu
def test_gpu_decrypt_legacy_key_fallback():
    """Records written under the legacy key SHA-256("Password") (EncryptUtils.java:50) decrypt
    through the fallback, on the host form and in the device form's second pass."""
    import torch

    from sdfs_amd.aes import LEGACY_KEY

    key = _key(32, 4)
    c, old = ciph(key), ciph(LEGACY_KEY)
    iv = bytes(range(7, 23))
    datas = [C.synth(9, i, 0, n).tobytes() for i, n in enumerate([0, 1, 15, 16, 100, 4096, 33000, 777] * 6)]
    cts = [(old if i % 3 == 0 else c).encryptCBC(d, iv) for i, d in enumerate(datas)]
    for i, (d, ct) in enumerate(zip(datas, cts)):
        assert c.decryptCBC(ct, iv) == d, i
    bad = bytearray(cts[4])
    bad[-1] ^= 0x33
    want_bad = _oracle_decrypt_with_fallback(key, iv, bytes(bad))
    if want_bad is None:
        with pytest.raises(IOError):
            c.decryptCBC(bytes(bad), iv)
    cts[4] = bytes(bad)
    # device form: all records in one buffer, fallback pass for the legacy ones
    dev = torch.device("cuda:0")
    src_off = np.concatenate([[0], np.cumsum([len(x) + 16 for x in cts[:-1]])]).astype(np.int64)
    buf = np.zeros(int(src_off[-1]) + len(cts[-1]) + 16, np.uint8)
    for o, x in zip(src_off, cts):
        buf[int(o): int(o) + len(x)] = np.frombuffer(x, np.uint8)
    dst_off = src_off.copy()
    out = torch.zeros(len(buf), dtype=torch.uint8, device=dev)
    plen = torch.zeros(len(cts), dtype=torch.int32, device=dev)
    c.decrypt_device(torch.from_numpy(buf).to(dev), torch.from_numpy(src_off).to(dev),
                     torch.tensor([len(x) for x in cts], dtype=torch.int32, device=dev), out,
                     torch.from_numpy(dst_off).to(dev), plen, iv=iv, legacy_fallback=True)
    torch.cuda.synchronize()
    o, pl = out.cpu().numpy(), plen.cpu().numpy().view(np.uint32)
    for i, ct in enumerate(cts):
        want = _oracle_decrypt_with_fallback(key, iv, ct)
        if want is None:
            assert pl[i] == 0xFFFFFFFF, i
        else:
            assert pl[i] == len(want) and o[dst_off[i]: dst_off[i] + pl[i]].tobytes() == want, i


@pytest.mark.gpu
def test_gpu_lz4_then_aes_chain():
    """Compressed + encrypted chunk store: AES of the framed LZ4 record, all on the device."""
    import torch

    from sdfs_amd.lz4 import HipLz4Compressor

    key, iv = _key(32, 3), bytes(16)
    c = ciph(key)
    z = HipLz4Compressor()
    n = 200
    lens = np.random.default_rng(13).integers(4096, 32769, n).astype(np.int64)
    src_off = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.int64)
    data = np.concatenate([Z.text_like(1, i, int(L)) for i, L in enumerate(lens)])
    dev = torch.device("cuda:0")
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)  # noqa: E731
    zroom = lens + lens // 255 + 20
    zoff = np.concatenate([[0], np.cumsum(zroom[:-1])]).astype(np.int64)
    zout = torch.zeros(int(zroom.sum()), dtype=torch.uint8, device=dev)
    zlen = torch.zeros(n, dtype=torch.int32, device=dev)
    z.compress_device(t(data, torch.uint8), t(src_off, torch.int64), t(lens, torch.int32), zout,
                      t(zoff, torch.int64), zlen, framed=True)
    aroom = zroom + 16
    aoff = np.concatenate([[0], np.cumsum(aroom[:-1])]).astype(np.int64)
    aout = torch.zeros(int(aroom.sum()), dtype=torch.uint8, device=dev)
    alen = torch.zeros(n, dtype=torch.int32, device=dev)
    c.encrypt_device(zout, t(zoff, torch.int64), zlen, aout, t(aoff, torch.int64), alen, iv=iv)
    torch.cuda.synchronize()
    a, al = aout.cpu().numpy(), alen.cpu().numpy()
    for i in range(0, n, 3):
        rec = Z.compress_framed(data[src_off[i]: src_off[i] + lens[i]])
        want = A.cbc_encrypt(key, iv, rec)
        assert a[aoff[i]: aoff[i] + al[i]].tobytes() == want, i
    z.destroy()


_VARIANT_CHECK = r"""
import os, struct, sys
import numpy as np
sys.path.insert(0, os.environ["ROOT"])
from oracle import aes_oracle as A
from oracle import cdc_oracle as C
from sdfs_amd.aes import HipEncryptUtils
from tests.test_aes import LENS, _key
for variant in (0, 3, 6, 7):
    os.environ["SDFS_AES_VARIANT"] = str(variant)  # read at create (tuning library only)
    key = _key(32, 9)
    c = HipEncryptUtils(key)
    rng = np.random.default_rng(20 + variant)
    lens = [int(x) for x in rng.integers(0, 34000, 300)] + LENS
    datas = [C.synth(8, i, 0, n).tobytes() for i, n in enumerate(lens)]
    offs = np.concatenate([[0], np.cumsum([len(d) + 1 for d in datas[:-1]])]).astype(np.uint64)
    base = np.zeros(int(offs[-1]) + len(datas[-1]) + 8, np.uint8)
    for o, d in zip(offs, datas):
        base[int(o): int(o) + len(d)] = np.frombuffer(d, np.uint8)
    iv = bytes(range(50, 66))
    for prefix in (None, -1):
        pre = b"" if prefix is None else struct.pack(">i", prefix)
        outs = c.encrypt_chunks(base, offs, lens, iv, nz_prefix=prefix)
        for d, out in zip(datas, outs):
            assert out == A.cbc_encrypt(key, iv, d, prefix=pre), variant
    c.destroy()
print("variants ok")
"""


@pytest.mark.gpu
def test_gpu_encrypt_variants_agree():
    """Every measured kernel layout (table copies, lane-per-record or quad-per-record; DESIGN.md
    §13) gives the oracle's bytes.  The layouts other than the production one exist only in the
    tuning library (the product library reads no environment), so this runs in a child process
    bound to it."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, ROOT=root, SDFS_CDC_LIB=_lib.TUNING_LIB)
    r = subprocess.run([sys.executable, "-c", _VARIANT_CHECK], capture_output=True, text=True, env=env,
                       timeout=240, cwd=root)
    assert r.returncode == 0 and "variants ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


@pytest.mark.gpu
def test_gpu_store_record_round_trip_on_device():
    """The stored-record chain both ways in HBM: chunk -> LZ4 putChunk record -> AES-CBC, then
    AES-CBC decrypt -> record decode -> the original chunk bytes (HashBlobArchive.putChunk /
    getChunk with compression and encryption on)."""
    import torch

    from sdfs_amd.lz4 import HipLz4Compressor

    key, iv = _key(32, 11), bytes(range(16))
    c = ciph(key)
    z = HipLz4Compressor()
    rng = np.random.default_rng(52)
    n = 500
    lens = rng.integers(0, 33000, n).astype(np.int64)
    kinds = [Z.text_like, Z.mixed]
    datas = [kinds[i % 2](3, i, int(L)) if L else np.zeros(0, np.uint8) for i, L in enumerate(lens)]
    src_off = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.int64)
    data = np.concatenate(datas) if lens.sum() else np.zeros(1, np.uint8)
    dev = torch.device("cuda:0")
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)  # noqa: E731
    d_data, d_soff, d_slen = t(data, torch.uint8), t(src_off, torch.int64), t(lens, torch.int32)
    zroom = lens + lens // 255 + 20
    zoff = np.concatenate([[0], np.cumsum(zroom[:-1])]).astype(np.int64)
    zout = torch.zeros(int(zroom.sum()), dtype=torch.uint8, device=dev)
    zlen = torch.zeros(n, dtype=torch.int32, device=dev)
    z.compress_device(d_data, d_soff, d_slen, zout, t(zoff, torch.int64), zlen, framed=True)
    aroom = zroom + 16
    aoff = np.concatenate([[0], np.cumsum(aroom[:-1])]).astype(np.int64)
    aout = torch.zeros(int(aroom.sum()), dtype=torch.uint8, device=dev)
    alen = torch.zeros(n, dtype=torch.int32, device=dev)
    c.encrypt_device(zout, t(zoff, torch.int64), zlen, aout, t(aoff, torch.int64), alen, iv=iv)
    # read side
    plain = torch.zeros_like(zout)
    plen = torch.zeros(n, dtype=torch.int32, device=dev)
    c.decrypt_device(aout, t(aoff, torch.int64), alen, plain, t(zoff, torch.int64), plen, iv=iv)
    back = torch.zeros(max(int(lens.sum()), 1) + 64, dtype=torch.uint8, device=dev)
    blen = torch.zeros(n, dtype=torch.int32, device=dev)
    z.decompress_device(plain, t(zoff, torch.int64), plen, back, d_soff, d_slen, blen, framed=True)
    torch.cuda.synchronize()
    assert torch.equal(plen, zlen)
    assert torch.equal(blen, d_slen)
    assert torch.equal(back[:int(lens.sum())], d_data[:int(lens.sum())])
    z.destroy()
